set -e
cd /root/repo
mkdir -p gpurun_out/flat
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tiers.py > gpurun_out/flat/parity.log 2>&1
for sh in reorder spaced escaped compact; do
  timeout -k 10 200 python tools/bench_extra.py general --shape $sh --steps 5 > gpurun_out/flat/gen_$sh.json 2> gpurun_out/flat/gen_$sh.err
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-extras > gpurun_out/flat/bench_$i.json 2> gpurun_out/flat/bench_$i.err
done
