set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/seg; mkdir -p $OUT
for r in 1 2; do
for s in 12500000 25000000; do
  timeout -k 10 200 python -u tools/bench_extra.py tbl --steps 20 --segment $s > $OUT/tbl_${s}_$r.json 2> $OUT/tbl_${s}_$r.err
  python -c "import json;d=json.load(open('$OUT/tbl_${s}_$r.json'));print('tbl $s', round(d['events_per_s']/1e9,3), d['check']['truth_mismatched_cells'])"
done
for s in 12500000 16666667; do
  timeout -k 10 300 python -u tools/bench_extra.py config3 --steps 20 --segment $s > $OUT/c3_${s}_$r.json 2> $OUT/c3_${s}_$r.err
  python -c "import json;d=json.load(open('$OUT/c3_${s}_$r.json'));print('c3 $s', round(d['events_per_s']/1e9,3), d['path_avg_ms'], d['check']['truth_mismatched_cells'])"
done
done
