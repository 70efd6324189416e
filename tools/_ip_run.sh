set -e
cd /root/repo
mkdir -p gpurun_out/ip4; rm -f gpurun_out/ip4/*
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiers.py > gpurun_out/ip4/tests.log 2>&1
