# stream rate with the copy kernel at raised wave priority, 1 GPU
set -o pipefail
out=gpurun_out/${1:-r6h}
mkdir -p $out
R=streaming-benchmarks_amd/bin/ysb_topology
for p in 0 1 0 1; do
  YSB_H2D_PRIO=$p timeout -k 10 200 $R --stream --sink none --seconds 10 --event-rate 6285714 --speedup 35 > $out/p$p.json 2> $out/p$p.err || exit 2
  python -c "import json; r=json.loads(open('$out/p$p.json').read().strip().splitlines()[-1]); print('prio', $p, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'])"
done
