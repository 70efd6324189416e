#!/bin/bash
# Round 3: record-mode overlap with stream priorities (scan stream greatest, count stream least)
# vs serial, config 3; and the .tbl tile-flags variant vs the production .tbl stage 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3p}; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for ov in 0 1; do
    YSB_REC_PRIO=1 YSB_REC_OVERLAP=$ov timeout -k 10 200 python3 tools/extra_one.py config3 > $O/c3_ov${ov}_$i.json 2> $O/c3_ov${ov}_$i.err || { tail -20 $O/c3_ov${ov}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c3_ov${ov}_$i.json')); print('prio ov=$ov', d['events_per_s']/1e9, d['ms_per_step'], d['avg_launch_ms'], d['avg_path_ms'], d['hbm_frac'], d['check']['truth_mismatched_cells'])"
  done
done
YSB_LIB_VARIANT=tflags timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_topology.py tests/test_gpu_tiers.py -k "tbl" > $O/tflags_tests.log 2>&1 || { tail -30 $O/tflags_tests.log; exit 1; }
tail -1 $O/tflags_tests.log
for v in base tflags base tflags base tflags; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 tools/extra_one.py tbl > $O/tbl_$v.json 2> $O/tbl_$v.err || { tail -20 $O/tbl_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/tbl_$v.json')); print('$v', round(d['events_per_s']/1e9,3), d['avg_launch_ms'], d['hbm_frac'], d['check']['truth_mismatched_cells'], d['check']['deferred'])"
done
