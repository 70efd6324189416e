#!/bin/bash
# round-4: learned-order vocabulary naming (parity + the two reordered legs), then the r4d diagnostics
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tiers.py tests/test_gpu_mutations.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 tools/extra_one.py reorder > $O/reorder.json 2> $O/reorder.err || exit 1
timeout -k 10 200 python3 tools/extra_one.py config3_reorder > $O/config3_reorder.json 2> $O/config3_reorder.err || exit 1
timeout -k 10 200 python3 tools/extra_one.py mixed > $O/mixed.json 2> $O/mixed.err || exit 1
timeout -k 10 200 python3 tools/extra_one.py reorder_flat_fixed > $O/reorder_flat_fixed.json 2> $O/reorder_flat_fixed.err || exit 1
cat $O/reorder.json $O/config3_reorder.json $O/mixed.json $O/reorder_flat_fixed.json
bash tools/ab/r4d.sh
