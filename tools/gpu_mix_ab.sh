# round 5 A/B: Kernel 1m (four-wave workgroups dealing lines by producer class) for layout 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5mix}; mkdir -p $O
export YSB_LIB_VARIANT=mix
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_tiers.py > $O/tests_tiers_mix.log 2>&1 || { tail -30 $O/tests_tiers_mix.log; exit 1; }
tail -1 $O/tests_tiers_mix.log
timeout -k 10 400 python3 -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mutations.py > $O/tests_more_mix.log 2>&1 || { tail -30 $O/tests_more_mix.log; exit 1; }
tail -1 $O/tests_more_mix.log
unset YSB_LIB_VARIANT
LEGS="mixed mixed_flat_fixed reorder_flat_fixed" TESTS=0 bash tools/ab_flat.sh ${1:-r5mix} base mix
