# mapped tests + the three replay modes, 1 GPU
set -o pipefail
out=gpurun_out/${1:-r6k}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mapped.py tests/test_gpu_topology.py -x -v --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
grep -c PASSED $out/tests.log
for m in mapped mapped-raw mapped copy; do
  timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 --replay $m > $out/$m.json 2> $out/$m.err || exit 2
  python -c "import json; r=json.load(open('$out/$m.json')); print('$m', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'], r['exact_vs_generator_truth'], r['get_stats']['p50_ms'], r['get_stats']['p99_ms'])"
done
