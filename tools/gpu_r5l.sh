set -o pipefail
mkdir -p gpurun_out/r5l
timeout -k 10 300 python tools/zerocopy_probe.py > gpurun_out/r5l/zc.json 2> gpurun_out/r5l/zc.err
echo rc=$?
