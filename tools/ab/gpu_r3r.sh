#!/bin/bash
# Round 3: (1) YSB_F_FLAT_FIRST takes a learned key order -- tier / parity tests, reordered-keys
# legs; (2) count kernel reading its runs 32 threads per slice (no search) -- record tests,
# config-3 A/B vs the search (oldcount); (3) Phase-A-only diagnostic timing of .tbl and JSON.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3r}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_tiers.py tests/test_gpu_parity.py tests/test_gpu_records.py tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for leg in reorder_flat reorder_flat_fixed reorder; do
  timeout -k 10 200 python3 tools/extra_one.py $leg > $O/$leg.json 2> $O/$leg.err || { tail -20 $O/$leg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$leg.json')); print('$leg', round(d['events_per_s']/1e9,3), d['kernel'], d['hbm_frac'], d['check']['truth_mismatched_cells'], d['check']['deferred'])"
done
for v in base oldcount base oldcount; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 tools/extra_one.py config3 > $O/c3_$v.json 2> $O/c3_$v.err || { tail -20 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$v.json')); print('c3 $v', round(d['events_per_s']/1e9,3), d['ms_per_step'], d['avg_launch_ms'], d['avg_path_ms'], d['hbm_frac'], d['check']['truth_mismatched_cells'])"
done
unset YSB_LIB_VARIANT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3trace -o run -- python3 tools/extra_one.py config3 > $O/c3trace.json 2> $O/c3trace.err || exit 1
export YSB_LIB_VARIANT=diag
for leg in tbl reorder_fixed; do
  timeout -k 10 200 python3 tools/extra_one.py $leg > $O/diag_$leg.json 2> $O/diag_$leg.err || { tail -20 $O/diag_$leg.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/diag_$leg.json')); print('diag $leg', d['avg_launch_ms'], d['bytes_per_event'], d['events'])"
done
