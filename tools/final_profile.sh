#!/bin/bash
# Round-end profiling of the headline (run on the GPU box via gpurun):
#   kernel trace + stats of the bench command, the timed launches of the scan kernel,
#   and separate --pmc FETCH_SIZE / WRITE_SIZE passes (traffic).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-final}
mkdir -p "$OUT"
BENCH="bench.py --steps 20 --warmup 10 --no-cpu --no-check --no-extras --no-live-traffic"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace.json"
python3 tools/timed_launches.py "$OUT/trace/run_kernel_trace.csv" "scan_kernel<false, false, false, 0>" 10 20 > "$OUT/scan_launches.txt"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-check --no-extras --no-live-traffic > "$OUT/pmc_fetch.json"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-check --no-extras --no-live-traffic > "$OUT/pmc_write.json"
timeout -k 10 600 python3 bench.py --extras-out "$OUT/bench_extras.json" > "$OUT/bench.json" 2> "$OUT/bench.err"
