#!/bin/bash
# Round 3: cache-resident join table as hash-and-displace (one slot per key; default) vs the
# two-choice cuckoo (YSB_CHD=0) -- parity / tier / mutation / topology tests, .tbl and
# headline A/B pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3c}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tiers.py tests/test_gpu_mutations.py tests/test_gpu_topology.py tests/test_gpu_segments.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
for v in base cuckoo; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 tools/extra_one.py tbl > $O/tbl_${v}_$i.json 2> $O/tbl_${v}_$i.err || { tail -20 $O/tbl_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/tbl_${v}_$i.json')); print('tbl $v', round(d['events_per_s']/1e9,3), d['avg_launch_ms'], d['hbm_frac'], d['check']['truth_mismatched_cells'], d['check']['deferred'])"
  timeout -k 10 200 python3 bench.py --no-cpu --no-check --no-extras > $O/h_${v}_$i.json 2> $O/h_${v}_$i.err || { tail -20 $O/h_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/h_${v}_$i.json')); print('headline $v', round(d['value']/1e9,3), d['roofline']['avg_launch_ms'])"
done
done
