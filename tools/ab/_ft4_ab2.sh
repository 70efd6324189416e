set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ft4b; mkdir -p $OUT
for r in 1 2 3 4; do
  for v in ft4 base; do
    if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-extras > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err
    python3 -c "import json;b=json.load(open('$OUT/b_${v}_$r.json'));print('$v', round(b['value']/1e9,3), b['roofline']['avg_launch_ms'])"
  done
done
