#!/bin/bash
# Round-end evidence on the shipped tree (GPU box), in two gpurun calls (each under 20 min):
#   tools/round_final.sh TAG a   smoke, the GPU suite, the headline's kernel trace + timed
#                                launches + PMC traffic passes and the full bench line
#                                (tools/final_profile.sh)
#   tools/round_final.sh TAG b   configs[2] / raw drop-in / mixed / native streaming traces and
#                                traffic (tools/round_profile.sh), the exchange cost with its
#                                kernel trace, SQ counters of the flat tier and the mixed interleave
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-final}; O=gpurun_out/$T; mkdir -p $O
if [ "${2:-a}" = a ]; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  bash tools/final_profile.sh $T || exit 1
  echo "round final a done"
else
  bash tools/round_profile.sh $T || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xtrace -o run -- python3 tools/exchange_cost.py --steps 10 --warmup 3 > $O/xtrace.json 2> $O/xtrace.err || exit 1
  timeout -k 10 300 python3 tools/exchange_cost.py --steps 20 --warmup 3 > $O/xcost.json 2> $O/xcost.err || exit 1
  OUT=$O/sq_flat CMD="tools/extra_one.py reorder_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
  OUT=$O/sq_mix CMD="tools/extra_one.py mixed_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
  echo "round final b done"
fi
