#!/bin/bash
# Round 3: record staging in one pass when a tile has <= 33 records (base) vs two half-wave passes (twopass) -- record / stream /
# rank / mutation tests with it, then config-3 A/B pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3b}; mkdir -p $O
unset YSB_LIB_VARIANT
timeout -k 10 400 python -u -m pytest tests/test_gpu_records.py tests/test_gpu_stream.py tests/test_gpu_ranks.py tests/test_gpu_mutations.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
echo "onepass $(tail -1 $O/t.log)"
for i in 1 2 3; do
for v in base twopass; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 tools/extra_one.py config3 > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || { tail -20 $O/c3_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_${v}_$i.json')); print('c3 $v', round(d['events_per_s']/1e9,3), d['avg_launch_ms'], d['avg_path_ms'], d['hbm_frac'], d['check']['truth_mismatched_cells'])"
done
done
