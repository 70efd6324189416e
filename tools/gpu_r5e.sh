set -o pipefail
mkdir -p gpurun_out/r5e
for k in 1 2; do
  timeout -k 10 120 python tools/h2d_probe.py > gpurun_out/r5e/probe_a$k.json 2> gpurun_out/r5e/probe_a$k.err || exit 1
  timeout -k 10 300 python tools/h2d_diag.py --events 30000000 > gpurun_out/r5e/diag_$k.json 2> gpurun_out/r5e/diag_$k.err || exit 1
  timeout -k 10 120 python tools/h2d_probe.py > gpurun_out/r5e/probe_b$k.json 2> gpurun_out/r5e/probe_b$k.err || exit 1
done
