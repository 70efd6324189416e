#!/bin/bash
# Round 3: one extra field per line through the flat tier -- tier / parity / mutation GPU
# tests, then the general-path bench with the extra-field shape (flat-first and fixed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3y}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiers.py tests/test_gpu_parity.py tests/test_gpu_mutations.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for h in flat none; do
  timeout -k 10 200 python3 tools/bench_extra.py general --shape extra --hint $h --steps 10 > $O/extra_$h.json 2> $O/extra_$h.err || { tail -20 $O/extra_$h.err; exit 1; }
  echo "hint $h: $(cat $O/extra_$h.json)"
done
