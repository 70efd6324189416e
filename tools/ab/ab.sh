#!/bin/bash
# A/B timing of library variants on the GPU box (never used for results):
#   tools/ab.sh TAG base VARIANT...   (base = lib/libysb_hip.so; others lib/libysb_hip_<v>.so)
# Each variant: the GPU parity tests, then the bench line with its extras (configs[2],
# .tbl), generator-truth checks on.  TESTS=0 skips the parity tests.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      > "$OUT/test_$v.log" 2>&1
  fi
  timeout -k 10 300 python -u bench.py --no-cpu --steps 20 ${BENCH_ARGS:-} > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"
  python - "$OUT/bench_$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); v = sys.argv[2]
x = d.get("extras") or {}
print(v, "json %.3f G %.4f %.4f ms mism %d" % (d["value"] / 1e9, d["roofline"]["frac"], d["roofline"]["avg_launch_ms"],
                                             (d["check"] or {}).get("truth_mismatched_cells", -1)),
      " ".join("| %s %.3f G %.4f ms mism %d" % (k, e["events_per_s"] / 1e9, e["avg_launch_ms"],
                                               e["check"]["truth_mismatched_cells"]) for k, e in x.items()))
PY
done
