#!/bin/bash
# Round 3: .tbl -- static s_setprio off (noprio), diagnostic splits (Phase A only: diag; no
# probe: dnoprobe, results wrong by design), two passes each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3v}; mkdir -p $O
for i in 1 2; do
for v in base noprio diag dnoprobe; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 tools/extra_one.py tbl > $O/tbl_${v}_$i.json 2> $O/tbl_${v}_$i.err || { tail -20 $O/tbl_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/tbl_${v}_$i.json')); print('tbl $v', round(d['events_per_s']/1e9,3), d['avg_launch_ms'], d['hbm_frac'], d['check']['truth_mismatched_cells'])"
done
done
