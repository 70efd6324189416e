#!/bin/bash
# A/B of general-path (flat tier) variants (never used for results): parity + tier tests on
# the current build, then tools/bench_extra.py general (reorder / spaced) and the headline
# bench line for each variant.   tools/ab_general.sh TAG base old VARIANT...
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_tiers.py > "$OUT/tests.log" 2>&1
echo tests ok
for v in "$@"; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  line="$v"
  for sh in reorder spaced; do
    timeout -k 10 200 python -u tools/bench_extra.py general --shape $sh --steps 20 > "$OUT/g_${sh}_$v.json" 2> "$OUT/g_${sh}_$v.err"
    line="$line $sh $(python -c "import json;d=json.load(open('$OUT/g_${sh}_$v.json'));print(round(d['events_per_s']/1e9,3), d['device_ms_per_step'], d['exact_vs_oracle'])")"
  done
  timeout -k 10 300 python -u bench.py --no-cpu --no-extras --steps 20 --warmup 10 > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
  line="$line head $(python -c "import json;b=json.load(open('$OUT/b_$v.json'));print(round(b['value']/1e9,3), b['roofline']['frac'])")"
  echo "$line"
done
