set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/hash
for v in base hl base hl base hl; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python -u tools/bench_extra.py tbl --steps 20 --segment 25000000 > gpurun_out/hash/tbl_$v.json 2> gpurun_out/hash/tbl_$v.err
  python -c "import json;d=json.load(open('gpurun_out/hash/tbl_$v.json'));print('$v', round(d['events_per_s']/1e9,3), d.get('scan_avg_launch_ms'), d['check']['truth_mismatched_cells'])"
done
