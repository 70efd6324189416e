#!/bin/bash
# Round 3: tiles of long lines staged up to capacity (lines inside parsed, the rest deferred)
# vs deferred whole (notrunc) -- tier / parity / mutation tests, the extra-field shape, and
# headline A/B pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3z}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiers.py tests/test_gpu_parity.py tests/test_gpu_mutations.py tests/test_gpu_segments.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in base notrunc; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 tools/bench_extra.py general --shape extra --hint flat --steps 10 > $O/extra_$v.json 2> $O/extra_$v.err || { tail -20 $O/extra_$v.err; exit 1; }
  echo "extra $v: $(cat $O/extra_$v.json)"
done
for i in 1 2 3; do
for v in base notrunc; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  timeout -k 10 200 python3 bench.py --no-cpu --no-check --no-extras > $O/h_${v}_$i.json 2> $O/h_${v}_$i.err || { tail -20 $O/h_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/h_${v}_$i.json')); print('headline $v', round(d['value']/1e9,3), d['roofline']['avg_launch_ms'])"
done
done
