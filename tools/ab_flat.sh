#!/bin/bash
# A/B of library variants on the flat-tier legs (mixed producers; reordered keys through the
# flat tier): tools/ab_flat.sh TAG base VARIANT...  (lib/libysb_hip_<v>.so, make variant)
# Each variant: the tier parity tests, then the two legs twice (interleaved).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for v in "$@"; do
  if [ $v = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  [ "${TESTS:-1}" = 0 ] && [ $v != base ] && continue   # TESTS=0: the parity tests for base only
  timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tiers.py > $O/tests_$v.log 2>&1 || { echo "$v tests FAILED"; tail -20 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
done
for r in 1 2; do
  for v in "$@"; do
    if [ $v = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
    for leg in ${LEGS:-mixed reorder_flat_fixed}; do
      timeout -k 10 200 python3 tools/extra_one.py $leg > $O/${leg}_${v}_$r.json 2> $O/${leg}_${v}_$r.err || exit 1
      python3 -c "import json;d=json.load(open('$O/${leg}_${v}_$r.json'));print('$v $leg', round(d['events_per_s']/1e9,3), d['hbm_frac'], d['avg_launch_ms'], d['check']['truth_mismatched_cells'], d['check']['deferred'])"
    done
  done
done
