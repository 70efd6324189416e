#!/bin/bash
# tools/extra_round.sh TAG: config 3, host-staged (PCIe) and streaming measurements.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/bench_extra.py config3 > "$OUT/config3.json" 2> "$OUT/config3.err"
timeout -k 10 120 python -u tools/bench_extra.py pcie --seconds 8 > "$OUT/pcie.json" 2> "$OUT/pcie.err"
timeout -k 10 200 python -u tools/bench_extra.py stream --rate 1000000 --seconds 25 > "$OUT/stream.json" 2> "$OUT/stream.err"
cat "$OUT"/*.json
