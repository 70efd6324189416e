set -e
cd /root/repo
mkdir -p gpurun_out/c3h; rm -f gpurun_out/c3h/*
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_records.py > gpurun_out/c3h/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python tools/bench_extra.py config3 --steps 20 --warmup 10 > gpurun_out/c3h/c3_$i.json 2> gpurun_out/c3h/c3_$i.err
done
