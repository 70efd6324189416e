set -o pipefail
mkdir -p gpurun_out/r5n
for k in 1 2; do
timeout -k 10 300 python tools/h2d_diag.py --zc --events 30000000 > gpurun_out/r5n/diag_$k.json 2> gpurun_out/r5n/diag_$k.err || exit 1
done
