set -e
cd /root/repo
mkdir -p gpurun_out/ip5; rm -f gpurun_out/ip5/*
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiers.py tests/test_gpu_parity.py > gpurun_out/ip5/tests.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 10 --no-cpu > gpurun_out/ip5/bench.json 2> gpurun_out/ip5/bench.err
