#!/bin/bash
# round-4 A/B: flat_parse_bl (base) against flat_parse_lds alone (nobl) on the flat-tier legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tiers.py tests/test_gpu_parity.py tests/test_gpu_mutations.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in base nobl base nobl; do
  if [ $v = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  for leg in mixed reorder_flat_fixed; do
    timeout -k 10 200 python3 tools/extra_one.py $leg > $O/${leg}_$v.json 2> $O/${leg}_$v.err || exit 1
    python3 -c "import json;d=json.load(open('$O/${leg}_$v.json'));print('$v $leg', round(d['events_per_s']/1e9,3), d['hbm_frac'], d['avg_launch_ms'], d['check']['truth_mismatched_cells'], d['check']['deferred'])"
  done
done
