#!/bin/bash
# round-4 diagnostics: the exchange's kernels (trace), SQ counters of the mixed-layout and
# flat-tier legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xtrace -o run -- python3 tools/exchange_cost.py --steps 10 --warmup 3 > $O/xtrace.json 2> $O/xtrace.err || exit 1
OUT=$O/mix CMD="tools/extra_one.py mixed_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
OUT=$O/flat CMD="tools/extra_one.py reorder_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
echo done
