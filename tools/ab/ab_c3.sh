#!/bin/bash
# config-3 timing of library variants (tools/bench_extra.py config3), never used for results
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u tools/bench_extra.py config3 --steps 3 > "$OUT/c3_$v.json" 2> "$OUT/c3_$v.err"
  python -c "import json;d=json.load(open('$OUT/c3_$v.json'));print('$v', round(d['events_per_s']/1e9,3), d['scan_avg_launch_ms'], d['check']['truth_mismatched_cells'])"
done
