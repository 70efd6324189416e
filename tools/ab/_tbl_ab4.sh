set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tbl4
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_topology.py -k "tbl" > gpurun_out/tbl4/tests.log 2>&1
echo tests ok
for v in base old base old base old; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python -u tools/bench_extra.py tbl --steps 20 --segment 25000000 > gpurun_out/tbl4/tbl_$v.json 2> gpurun_out/tbl4/tbl_$v.err
  python -c "import json;d=json.load(open('gpurun_out/tbl4/tbl_$v.json'));print('$v', round(d['events_per_s']/1e9,3), d.get('scan_avg_launch_ms'), d['check']['truth_mismatched_cells'])"
done
