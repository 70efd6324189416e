#!/bin/bash
# Instruction-cache counters (SQC_ICACHE_*, counted in the SQ block on gfx950: one pass of
# eight SQ counters) over one leg each: tools/icache_passes.sh TAG LEG...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/$1; shift; mkdir -p $O
for leg in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
    SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_IFETCH --output-format csv -d $O/ic_$leg -o run \
    -- python3 tools/extra_one.py $leg --extra-steps 2 --warmup 1 > $O/ic_$leg.json 2> $O/ic_$leg.err || { echo "$leg failed"; tail -5 $O/ic_$leg.err; exit 1; }
  echo "$leg done"
done
