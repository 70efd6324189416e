set -o pipefail
mkdir -p gpurun_out/r5h
for k in 1 2; do
for m in 0 1 2 3; do
  YSB_H2D_MODE=$m timeout -k 10 150 python tools/h2d_diag.py --pre none --events 40000000 > gpurun_out/r5h/m${m}_$k.json 2> gpurun_out/r5h/m${m}_$k.err || exit 1
done
done
