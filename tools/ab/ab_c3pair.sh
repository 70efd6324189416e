#!/bin/bash
# A/B of the config-3 path (never used for results): record-mode tests on the current
# build, then tools/bench_extra.py config3 for the current (base) and previous (old)
# builds, interleaved, with the kernel-stats split.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-c3pair}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_records.py > "$OUT/tests.log" 2>&1
echo tests ok
for r in 1 2; do
  for v in base old; do
    if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
    timeout -k 10 300 python -u tools/bench_extra.py config3 --steps 20 --warmup 10 > "$OUT/c3_${v}_$r.json" 2> "$OUT/c3_${v}_$r.err"
    python -c "import json;d=json.load(open('$OUT/c3_${v}_$r.json'));print('$v', round(d['events_per_s']/1e9,3), d['scan_avg_launch_ms'], d.get('path_ms', d.get('avg_path_ms')), d['check']['truth_mismatched_cells'])"
  done
done
