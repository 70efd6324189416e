# round 5: the flush row-cap test and the stream GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5y; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py > $O/tests.log 2>&1; rc=$?
tail -25 $O/tests.log; exit $rc
