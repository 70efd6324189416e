#!/bin/bash
# Round 3: YSB_F_FLAT_FIRST takes a learned key order -- tier / parity GPU tests, then the
# reordered-keys legs (hint, hint + fixed, no hint).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3q}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiers.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for leg in reorder_flat reorder_flat_fixed reorder; do
  timeout -k 10 200 python3 tools/extra_one.py $leg > $O/$leg.json 2> $O/$leg.err || { tail -20 $O/$leg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$leg.json')); print('$leg', round(d['events_per_s']/1e9,3), d['kernel'], d['hbm_frac'], d['check']['truth_mismatched_cells'], d['check']['deferred'])"
done
