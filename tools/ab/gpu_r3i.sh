# full GPU test suite (round 3, after the pipelined exchange)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3i; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
