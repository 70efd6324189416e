set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ffast; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiers.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1
echo tests ok
for sh in reorder spaced compact generator; do
  timeout -k 10 200 python -u tools/bench_extra.py general --shape $sh --hint flat --steps 20 > $OUT/g_${sh}.json 2> $OUT/g_${sh}.err
  python3 -c "import json;d=json.load(open('$OUT/g_${sh}.json'));print('$sh flat', round(d['events_per_s']/1e9,3), d['device_ms_per_step'], d['exact_vs_oracle'], d['deferred'])"
done
timeout -k 10 500 python -u bench.py --no-cpu --stream-seconds 0 > $OUT/bench.json 2> $OUT/bench.err
python3 -c "
import json;d=json.load(open('$OUT/bench.json'));print(d['value']/1e9, d['roofline']['frac'])
for k,e in d['extras'].items(): print(k, round(e.get('events_per_s',0)/1e9,3), e.get('avg_launch_ms'), e.get('hbm_frac'), e.get('check',{}).get('truth_mismatched_cells'), e.get('check',{}).get('deferred'))"
