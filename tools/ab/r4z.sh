#!/bin/bash
# round-4: the GPU suite with the 64-line sample and the per-tile dispatch; then base (layout 4
# for mixed batches) against m2 (the flat tier, layout 2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
TESTS=0 LEGS="mixed mixed_blocks reorder" bash tools/ab_flat.sh r4z base m2
