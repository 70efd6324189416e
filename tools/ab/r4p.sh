#!/bin/bash
# round-4: bl2 with both value checks and no branch (nb) against bl2; SQ of nb on the flat tier
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_flat.sh r4o base nb || exit 1
YSB_LIB_VARIANT=nb OUT=gpurun_out/r4o/flat_nb CMD="tools/extra_one.py reorder_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
echo done
