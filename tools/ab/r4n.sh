#!/bin/bash
# round-4: SQ counters of the flat tier (flat_parse_bl2), configs[2] and .tbl legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4n/flat CMD="tools/extra_one.py reorder_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
OUT=gpurun_out/r4n/c3 CMD="tools/extra_one.py config3 --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
OUT=gpurun_out/r4n/tbl CMD="tools/extra_one.py tbl --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
echo done
