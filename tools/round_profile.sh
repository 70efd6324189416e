#!/bin/bash
# Round-end evidence on the GPU box (gpurun), every GPU step under its own time limit and
# chained: the GPU tests, smoke, the headline's kernel trace (stats + timed launches) and
# FETCH_SIZE / WRITE_SIZE passes, config 3's kernel trace and traffic passes, then the
# driver's bench line.   tools/round_profile.sh TAG
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/${1:-r02c}
mkdir -p "$OUT"
export TMPDIR=/tmp
H="$R/bench.py --steps 20 --warmup 10 --no-cpu --no-check --no-extras"
C3="$R/tools/bench_extra.py config3 --steps 20 --warmup 10 --segment 16666667"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
echo "tests ok"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke ok"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $H > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
python3 $R/tools/timed_launches.py "$OUT/trace/run_kernel_trace.csv" "scan_kernel<false, false, false, 0>" 10 20 > "$OUT/scan_launches.txt"
echo "trace ok"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-check --no-extras > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-check --no-extras > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
python3 $R/tools/pmc_summary.py "$OUT" "scan_kernel<false, false, false, 0>" > "$OUT/pmc_summary.txt"
echo "pmc ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3trace" -o run -- python3 $C3 > "$OUT/c3_trace.json" 2> "$OUT/c3_trace.err"
python3 $R/tools/timed_launches.py "$OUT/c3trace/run_kernel_trace.csv" "scan_kernel<true, false, true, 0>" 10 20 > "$OUT/c3_scan_launches.txt"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/c3/pmc_fetch" -o run -- python3 $R/tools/bench_extra.py config3 --steps 2 --warmup 1 --segment 16666667 > "$OUT/c3_pmc_fetch.json" 2> "$OUT/c3_pmc_fetch.err"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c3/pmc_write" -o run -- python3 $R/tools/bench_extra.py config3 --steps 2 --warmup 1 --segment 16666667 > "$OUT/c3_pmc_write.json" 2> "$OUT/c3_pmc_write.err"
echo "c3 ok"
cd "$R"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
