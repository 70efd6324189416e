set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 200 python tools/h2d_probe.py --free-test > gpurun_out/r5j/free.json 2> gpurun_out/r5j/free.err
