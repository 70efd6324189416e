# A/B of the streaming feed's copy stream (diagnostic knobs YSB_SPLIT_STREAM / YSB_H2D_WG), 1 GPU
set -o pipefail
out=gpurun_out/${1:-r6c}
mkdir -p $out
for v in "0 1" "1 1" "0 2" "1 2" "0 1"; do
  set -- $v
  YSB_SPLIT_STREAM=$1 YSB_H2D_WG=$2 timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 > $out/s$1_w$2.json 2> $out/s$1_w$2.err || exit 2
  python -c "import json; r=json.load(open('$out/s$1_w$2.json')); print('split', $1, 'wg', $2, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['exact_vs_generator_truth'])"
done
timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 --batch-ms 200 > $out/b200.json 2> $out/b200.err || exit 3
python -c "import json; r=json.load(open('$out/b200.json')); print('batch 200', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['exact_vs_generator_truth'])"
