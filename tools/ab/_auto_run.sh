set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/auto; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiers.py > $OUT/tests.log 2>&1
echo tests ok
for sh in reorder compact generator; do
  timeout -k 10 200 python -u tools/bench_extra.py general --shape $sh --hint auto --steps 5 > $OUT/g_${sh}.json 2> $OUT/g_${sh}.err
  python3 -c "import json;d=json.load(open('$OUT/g_${sh}.json'));print('$sh auto', round(d['events_per_s_device']/1e9,3), round(d['events_per_s_pcie_inclusive']/1e9,3), d['exact_vs_oracle'], d['deferred'], d['launches'])"
done
