#!/bin/bash
# A/B timing of library variants on the GPU box (never used for results):
#   tools/ab.sh TAG base VARIANT...   (base = lib/libysb_hip.so; others lib/libysb_hip_<v>.so)
# Each variant: the GPU parity tests, then the bench line (generator-truth check on).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    > "$OUT/test_$v.log" 2>&1
  timeout -k 10 300 python -u bench.py --no-cpu --steps 20 ${BENCH_ARGS:-} > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"
  python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', round(d['value']/1e9,3), d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['check']['truth_mismatched_cells'], d['check']['deferred_to_general_path'])"
done
