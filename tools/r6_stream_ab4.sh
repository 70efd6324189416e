# stream copy rate vs the replay cycle's size (IOMMU / TLB reach?), 1 GPU; THP state
set -o pipefail
out=gpurun_out/${1:-r6f}
mkdir -p $out
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $out/thp.txt 2>&1
ls /sys/kernel/iommu_groups 2>/dev/null | wc -l >> $out/thp.txt
cat /sys/class/iommu/*/devices 2>/dev/null | head -2 >> $out/thp.txt
dmesg 2>/dev/null | grep -i -m3 iommu >> $out/thp.txt
for v in "6285714 35 100" "1257143 175 500" "314286 700 2000"; do
  set -- $v
  timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate $1 --speedup $2 --batch-ms $3 > $out/r$1.json 2> $out/r$1.err || exit 2
  python -c "import json; r=json.load(open('$out/r$1.json')); print('rate', $1, 'speedup', $2, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'], r['per_shard'][0]['replay_GB'], r['exact_vs_generator_truth'])"
done
cat $out/thp.txt
