set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/rep; mkdir -p $OUT
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-extras > $OUT/b$i.json 2> $OUT/b$i.err
  python3 -c "import json;d=json.load(open('$OUT/b$i.json'));print('head', round(d['value']/1e9,3), d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['check']['truth_mismatched_cells'])"
done
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/bench_extra.py config3 --steps 20 --warmup 10 --segment 16666667 > $OUT/c$i.json 2> $OUT/c$i.err
  python3 -c "import json;d=json.load(open('$OUT/c$i.json'));print('c3', round(d['events_per_s']/1e9,3), d['path_avg_ms'], d['check']['truth_mismatched_cells'])"
done
