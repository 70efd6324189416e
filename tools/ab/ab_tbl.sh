#!/bin/bash
# A/B of .tbl scan geometries (never used for results): tools/bench_extra.py tbl (with its
# generator-truth check) per library variant.   tools/ab_tbl.sh TAG base VARIANT...
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python -u tools/bench_extra.py tbl --steps 20 > "$OUT/tbl_$v.json" 2> "$OUT/tbl_$v.err"
  python -c "import json;d=json.load(open('$OUT/tbl_$v.json'));print('$v', round(d['events_per_s']/1e9,3), d.get('scan_avg_launch_ms'), d['check']['truth_mismatched_cells'])"
done
