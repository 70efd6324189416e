# round 5: bench.config3_ranks on a one-rank RCCL group
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5zb; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_ranks.py > $O/tests.log 2>&1; rc=$?
tail -25 $O/tests.log; exit $rc
