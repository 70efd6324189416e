set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ft4; mkdir -p $OUT
export YSB_LIB_VARIANT=ft4
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiers.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1
unset YSB_LIB_VARIANT
echo tests ok
for r in 1 2 3; do
  for v in base ft4; do
    if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-extras > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err
    timeout -k 10 200 python -u tools/bench_extra.py general --shape reorder --steps 20 > $OUT/g_${v}_$r.json 2> $OUT/g_${v}_$r.err
    python3 -c "import json;b=json.load(open('$OUT/b_${v}_$r.json'));g=json.load(open('$OUT/g_${v}_$r.json'));print('$v', round(b['value']/1e9,3), b['roofline']['avg_launch_ms'], 'reorder', round(g['events_per_s']/1e9,3), g['exact_vs_oracle'])"
  done
done
