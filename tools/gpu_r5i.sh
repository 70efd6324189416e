set -o pipefail
mkdir -p gpurun_out/r5i
(lspci -tv > gpurun_out/r5i/lspci_tv.txt 2>&1; rocm-smi --showtopo > gpurun_out/r5i/topo.txt 2>&1; rocm-smi --showbus > gpurun_out/r5i/bus.txt 2>&1) || true
for k in 1 2 3; do
  timeout -k 10 120 python tools/h2d_probe.py --thp > gpurun_out/r5i/thp_$k.json 2> gpurun_out/r5i/thp_$k.err || exit 1
done
