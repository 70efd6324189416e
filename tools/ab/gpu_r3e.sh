# learned key order (layout 3): tier tests, the layout extras, SQ counters of layout 3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_tiers.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for leg in reorder reorder_fixed compact; do timeout -k 10 300 python -u tools/extra_one.py $leg > $O/$leg.json 2> $O/$leg.err || exit 1; done
OUT=$O/sq CMD="tools/extra_one.py reorder --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
python3 tools/pmc_summary.py $O/sq "scan_kernel" | grep -E "SQ_INSTS_VALU|SQ_INSTS_SALU|SQ_INSTS_LDS |SQ_LDS_BANK|SQ_LDS_IDX|SQ_WAVE_CYCLES|SQ_INSTS_BRANCH"
python3 -c "
import json
for k in ('reorder','reorder_fixed','compact'):
    d=json.load(open('$O/%s.json'%k)); print(k, d['events_per_s']/1e9, d['hbm_frac'], d['kernel'], d['check']['truth_mismatched_cells'], d['check']['deferred'])
"
