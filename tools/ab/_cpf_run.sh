set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/cpf
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiers.py tests/test_gpu_parity.py > gpurun_out/cpf/tests.log 2>&1
echo tests ok
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/cpf/bench.json 2> gpurun_out/cpf/bench.err
python3 -c "
import json;d=json.load(open('gpurun_out/cpf/bench.json'));print(d['value']/1e9, d['roofline']['frac'])
for k,e in d['extras'].items(): print(k, round(e.get('events_per_s',0)/1e9,3), e.get('avg_launch_ms'), e.get('hbm_frac'), e.get('check',{}).get('truth_mismatched_cells'), e.get('check',{}).get('deferred'))"
