set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tbl2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_topology.py -k "tbl" > gpurun_out/tbl2/tests.log 2>&1
echo tests ok
bash tools/ab_tbl.sh tbl2 base old base old
bash tools/_tbl_sq.sh
