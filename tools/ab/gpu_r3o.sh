#!/bin/bash
# Round 3: record-mode overlap (partition + count beside the next scan) -- GPU tests, then
# config-3 A/B pairs YSB_REC_OVERLAP=0 / 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3o}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for i in 1 2; do
  for ov in 0 1; do
    YSB_REC_OVERLAP=$ov timeout -k 10 200 python3 tools/extra_one.py config3 > $O/c3_ov${ov}_$i.json 2> $O/c3_ov${ov}_$i.err || { tail -20 $O/c3_ov${ov}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c3_ov${ov}_$i.json')); print('ov=$ov', d['events_per_s']/1e9, d['ms_per_step'], d['avg_launch_ms'], d['avg_path_ms'], d['hbm_frac'], d['check'])"
  done
done
