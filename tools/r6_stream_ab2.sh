# A/B of the streaming feed after the copy queue's barrier skip, 1 GPU
set -o pipefail
out=gpurun_out/${1:-r6d}
mkdir -p $out
for v in "100 mapped" "200 mapped" "100 copy"; do
  set -- $v
  timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 --batch-ms $1 --replay $2 > $out/b$1_$2.json 2> $out/b$1_$2.err || exit 2
  python -c "import json; r=json.load(open('$out/b$1_$2.json')); print('batch', $1, '$2', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['exact_vs_generator_truth'])"
done
