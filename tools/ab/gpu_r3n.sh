# config-3 join table size: buckets per key x4 = 8 (production, 4 GiB), 4 (2 GiB), 2 (1 GiB), 1 (512 MiB)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_topology.py tests/test_gpu_records.py tests/test_gpu_stream.py -k "tbl or record or config3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in base bx4 bx2 bx1 base bx4 bx2 bx1; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u tools/extra_one.py config3 > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/c3_$v.json'));d=d.get('config3',d);print('$v', round(d['events_per_s']/1e9,3), d.get('scan_avg_launch_ms'), d.get('path_avg_ms'), d.get('hbm_frac'), d['check'].get('truth_mismatched_cells'))"
done
