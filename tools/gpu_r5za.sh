# round 5: the key table with the shift-xor slot -- tier / mutation / parity GPU tests, then the flat legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5za; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_tiers.py tests/test_gpu_mutations.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for leg in mixed reorder_flat_fixed; do
  timeout -k 10 200 python3 tools/extra_one.py $leg > $O/$leg.json 2> $O/$leg.err || exit 1
  python3 -c "import json;d=json.load(open('$O/$leg.json'));print('$leg', round(d['events_per_s']/1e9,3), d['hbm_frac'], d['check']['truth_mismatched_cells'], d['check']['deferred'])"
done
