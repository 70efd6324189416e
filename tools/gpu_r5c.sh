# H2D: per-stream (SDMA engine) rates and split copies, three fresh processes, then blit
# kernels instead of SDMA (HSA_ENABLE_SDMA=0).
set -o pipefail
mkdir -p gpurun_out/r5c
for k in 1 2 3; do
  timeout -k 10 120 python tools/h2d_probe.py --streams > gpurun_out/r5c/streams_$k.json 2> gpurun_out/r5c/streams_$k.err || { echo "probe $k rc=$?"; exit 1; }
done
HSA_ENABLE_SDMA=0 timeout -k 10 120 python tools/h2d_probe.py --streams > gpurun_out/r5c/blit.json 2> gpurun_out/r5c/blit.err
echo "blit rc=$?"
timeout -k 10 150 python tools/h2d_diag.py --pre none --events 30000000 > gpurun_out/r5c/pre_none.json 2> gpurun_out/r5c/pre_none.err
echo "diag rc=$?"
