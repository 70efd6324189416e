set -o pipefail
mkdir -p gpurun_out/r5d
for k in 1 2 3; do
  timeout -k 10 120 python tools/h2d_probe.py --streams > gpurun_out/r5d/streams_$k.json 2> gpurun_out/r5d/streams_$k.err || exit 1
  timeout -k 10 150 python tools/h2d_diag.py --pre none --events 30000000 > gpurun_out/r5d/pre_none_$k.json 2> gpurun_out/r5d/pre_none_$k.err || exit 1
done
