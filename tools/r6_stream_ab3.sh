# same-box: host_staged raw vs the stream at several batch sizes / flush periods, 1 GPU
set -o pipefail
out=gpurun_out/${1:-r6e}
mkdir -p $out
timeout -k 10 200 python -c "
import sys, json; sys.path[:0] = ['tools', 'streaming-benchmarks_amd']
import bench_dropin
r = bench_dropin.host_staged(0, 100_000_000, raw=True)
print(json.dumps(r))" > $out/host_staged.json 2> $out/host_staged.err || exit 1
python -c "import json; r=json.load(open('$out/host_staged.json')); print('host_staged raw', round(r['events_per_s']/1e6,1), r['h2d_GBs'], r['copy_busy_frac'], r['h2d_ms_per_batch'])"
for v in "100 1000" "300 1000" "100 100000"; do
  set -- $v
  timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 --batch-ms $1 --flush-ms $2 > $out/b$1_f$2.json 2> $out/b$1_f$2.err || exit 2
  python -c "import json; r=json.load(open('$out/b$1_f$2.json')); print('batch', $1, 'flush', $2, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'], r['exact_vs_generator_truth'])"
done
