#!/bin/bash
# Round 3: one-sweep partition (fixed-capacity runs, no histogram sweep) -- record tests with
# it, then config-3 A/B pairs vs the two-sweep partition.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3w}; mkdir -p $O
export YSB_LIB_VARIANT=onesweep
timeout -k 10 400 python -u -m pytest tests/test_gpu_records.py tests/test_gpu_stream.py tests/test_gpu_ranks.py -x -q --timeout 200 --timeout-method thread > $O/tests_onesweep.log 2>&1 || { tail -30 $O/tests_onesweep.log; exit 1; }
echo "onesweep $(tail -1 $O/tests_onesweep.log)"
for i in 1 2; do
for v in base onesweep; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 tools/extra_one.py config3 > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || { tail -20 $O/c3_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_${v}_$i.json')); print('c3 $v', round(d['events_per_s']/1e9,3), d['ms_per_step'], d['avg_launch_ms'], d['avg_path_ms'], round(d['avg_path_ms']-d['avg_launch_ms'],4), d['hbm_frac'], d['check']['truth_mismatched_cells'])"
done
done
