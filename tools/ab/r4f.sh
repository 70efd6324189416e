#!/bin/bash
# round-4: vectorized exchange pack/unpack/plan -- the exchange tests, then its cost
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ranks.py tests/test_gpu_group_host.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xtrace -o run -- python3 tools/exchange_cost.py --steps 10 --warmup 3 > $O/xtrace.json 2> $O/xtrace.err || exit 1
timeout -k 10 300 python3 tools/exchange_cost.py --steps 20 --warmup 3 > $O/xcost.json 2> $O/xcost.err || exit 1
tail -1 $O/xcost.json
