set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ff; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiers.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1
echo tests ok
for sh in reorder spaced compact generator; do
  for h in none flat; do
    timeout -k 10 200 python -u tools/bench_extra.py general --shape $sh --hint $h --steps 20 > $OUT/g_${sh}_$h.json 2> $OUT/g_${sh}_$h.err
    python3 -c "import json;d=json.load(open('$OUT/g_${sh}_$h.json'));print('$sh $h', round(d['events_per_s']/1e9,3), d['device_ms_per_step'], d['exact_vs_oracle'], d['deferred'])"
  done
done
timeout -k 10 200 python -u tools/bench_extra.py tbl --steps 20 --segment 25000000 > $OUT/tbl.json 2> $OUT/tbl.err
python3 -c "import json;d=json.load(open('$OUT/tbl.json'));print('tbl', round(d['events_per_s']/1e9,3), d['check']['truth_mismatched_cells'])"
