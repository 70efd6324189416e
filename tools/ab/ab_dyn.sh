#!/bin/bash
# A/B of the scan schedule (static share vs dynamic chunk claims) on the GPU box:
#   tools/ab_dyn.sh OUTDIR "PCT:CHUNK PCT:CHUNK ..."
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
for cfg in $2; do
  pct=${cfg%%:*}; ch=${cfg##*:}
  YSB_DYN_PCT=$pct YSB_DYN_CHUNK=$ch timeout -k 10 200 python -u bench.py --no-cpu --no-check --steps 20 \
    > "$OUT/bench_${pct}_${ch}.json" 2> "$OUT/bench_${pct}_${ch}.err"
  python -c "import json; d=json.load(open('$OUT/bench_${pct}_${ch}.json')); print('$cfg', round(d['value']/1e9,3), d['ms_per_step'])"
done
