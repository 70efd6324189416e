#!/bin/bash
# Round 3: partition kernel geometry A/B on config 3 -- slices per level-1 bin (32 / 64) and
# staged records per block (64 / 32: 72 KiB of LDS, two workgroups per CU); record tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3t}; mkdir -p $O
for v in base q64r32; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_records.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
done
for i in 1 2; do
for v in base q64r32 q64r64 q32r32; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 tools/extra_one.py config3 > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || { tail -20 $O/c3_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_${v}_$i.json')); print('c3 $v', round(d['events_per_s']/1e9,3), d['ms_per_step'], d['avg_launch_ms'], d['avg_path_ms'], round(d['avg_path_ms']-d['avg_launch_ms'],4), d['hbm_frac'], d['check']['truth_mismatched_cells'])"
done
done
