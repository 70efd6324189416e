# stream rate with / without the copy-timing markers, split on the copy stream / its own, 1 GPU
set -o pipefail
out=gpurun_out/${1:-r6g}
mkdir -p $out
R=streaming-benchmarks_amd/bin/ysb_topology
for v in "0 t" "0 n" "1 n" "0 t"; do
  set -- $v
  extra=""; [ "$2" = n ] && extra="--no-timing"
  YSB_SPLIT_STREAM=$1 timeout -k 10 200 $R --stream --sink none --seconds 10 --event-rate 6285714 --speedup 35 $extra > $out/s$1_$2.json 2> $out/s$1_$2.err || exit 2
  python -c "import json; r=json.loads(open('$out/s$1_$2.json').read().strip().splitlines()[-1]); print('split', $1, '$2', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'])"
done
