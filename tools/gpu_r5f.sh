# Hypothesis: ysb_submit's copy stream and compute stream share a hardware queue in some
# processes (GPU_MAX_HW_QUEUES=4 per process, streams assigned round robin).
set -o pipefail
mkdir -p gpurun_out/r5f
for k in 1 2 3; do
  timeout -k 10 150 python tools/h2d_diag.py --pre none --events 30000000 > gpurun_out/r5f/q4_$k.json 2> gpurun_out/r5f/q4_$k.err || exit 1
  GPU_MAX_HW_QUEUES=16 timeout -k 10 150 python tools/h2d_diag.py --pre none --events 30000000 > gpurun_out/r5f/q16_$k.json 2> gpurun_out/r5f/q16_$k.err || exit 1
done
timeout -k 10 300 python tools/h2d_diag.py --events 30000000 > gpurun_out/r5f/full_q4.json 2> gpurun_out/r5f/full_q4.err || exit 1
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python tools/h2d_diag.py --events 30000000 > gpurun_out/r5f/full_q16.json 2> gpurun_out/r5f/full_q16.err
