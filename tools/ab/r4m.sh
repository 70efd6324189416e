#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4m/mix CMD="tools/extra_one.py mixed_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
LEGS="mixed reorder_flat_fixed" bash tools/ab_flat.sh r4m base fs
