#!/bin/bash
# round-4: SQ counters of the flat-tier legs with flat_parse_bl
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4i/mix CMD="tools/extra_one.py mixed_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
OUT=gpurun_out/r4i/flat CMD="tools/extra_one.py reorder_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
echo done
