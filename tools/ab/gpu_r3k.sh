# .tbl bitmap diagnosis: full (base), Phase-A bitmap only (bmA), LDS reserve only (bmL), none (nobm)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3k3; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_topology.py tests/test_gpu_records.py -k "tbl" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
for v in base r64s r32 old bm base r64s r32 old bm; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python -u tools/bench_extra.py tbl --steps 20 > $O/tbl_$v.json 2> $O/tbl_$v.err || { tail -5 $O/tbl_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/tbl_$v.json'));print('$v', round(d['events_per_s']/1e9,3), d.get('scan_avg_launch_ms'), d.get('hbm_frac'), d['check']['truth_mismatched_cells'])"
done
