#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export YSB_LIB_VARIANT=t4b
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tiers.py tests/test_gpu_mutations.py > gpurun_out/r4za_tests.log 2>&1 || { tail -30 gpurun_out/r4za_tests.log; exit 1; }
tail -1 gpurun_out/r4za_tests.log
unset YSB_LIB_VARIANT
TESTS=0 LEGS="mixed mixed_blocks" bash tools/ab_flat.sh r4za base t4b m2
