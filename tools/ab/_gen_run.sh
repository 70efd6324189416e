set -e
cd /root/repo
mkdir -p gpurun_out/gen2; rm -f gpurun_out/gen2/*
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tiers.py > gpurun_out/gen2/tests.log 2>&1
for sh in escaped reorder; do
  timeout -k 10 200 python tools/bench_extra.py general --shape $sh --steps 5 > gpurun_out/gen2/gen_$sh.json 2> gpurun_out/gen2/gen_$sh.err
done
