#!/bin/bash
# Profiling passes for the scan kernel (run on the GPU box via gpurun).
#   tools/profile.sh trace        -> kernel trace + stats
#   tools/profile.sh pmc NAME CTRS -> one --pmc pass (separate run per counter group)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/prof}
mkdir -p "$OUT"
BENCH=${BENCH:-"bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu --no-check"}
case "$1" in
  trace)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace.json" ;;
  pmc)
    name=$2; shift 2
    timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$name" -o run -- python3 $BENCH > "$OUT/pmc_$name.json" ;;
  list)
    timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 ;;
esac
