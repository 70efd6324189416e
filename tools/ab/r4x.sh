#!/bin/bash
# round-4: per-tile dispatch (layout 4, base) against the flat tier for mixed batches (m2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mutations.py tests/test_gpu_raw.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
LEGS="mixed mixed_blocks" bash tools/ab_flat.sh r4x base m2
