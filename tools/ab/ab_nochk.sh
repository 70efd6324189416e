#!/bin/bash
# A/B timing only (no tests, no truth check): diagnostic builds whose results are wrong by design.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-check --steps 20 > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"
  python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', round(d['value']/1e9,3), d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
done
