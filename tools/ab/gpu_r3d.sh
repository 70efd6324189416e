#!/bin/bash
# Round 3: where config 3's scan time goes (diagnostic builds, counts wrong by design):
# no record staging (dnorec), no join probe (dnoprobe), neither (dnoboth).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3d}; mkdir -p $O
for i in 1 2; do
for v in base dnorec dnoprobe dnoboth; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 tools/extra_one.py config3 > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || { tail -20 $O/c3_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_${v}_$i.json')); print('c3 $v', round(d['events_per_s']/1e9,3), d['avg_launch_ms'], d['avg_path_ms'], d['check']['truth_mismatched_cells'])"
done
done
