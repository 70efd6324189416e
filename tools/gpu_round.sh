#!/bin/bash
# One GPU-box session: parity tests, the bench line, the rocprofv3 kernel-trace
# summary and the HBM PMC passes.  Every GPU step has its own time limit and the
# steps are chained: the first failure ends the script.
#   tools/gpu_round.sh TAG [tests|bench|trace|pmc ...]   (default: all four)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$PWD
TAG=${1:-r01}; shift || true
STAGES=${*:-tests bench trace pmc}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STAGES; do
  case $s in
    tests)
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    trace)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
         -d "$OUT/trace" -o run -- python3 "$REPO/bench.py" --steps 20 --warmup 10 --no-cpu --no-check \
         > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err") ;;
    pmc)
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv \
         -d "$OUT/pmc_fetch" -o run -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu --no-check \
         > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err")
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv \
         -d "$OUT/pmc_write" -o run -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu --no-check \
         > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err") ;;
    *) echo "unknown stage $s"; exit 2 ;;
  esac
  echo "stage $s ok"
done
