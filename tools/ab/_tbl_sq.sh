set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export OUT=gpurun_out/tblsq
export BENCH="tools/bench_extra.py tbl --steps 2 --warmup 1"
bash tools/pmc_sq.sh
python3 tools/pmc_summary.py gpurun_out/tblsq "scan_kernel<false, true, false>" > gpurun_out/tblsq/summary.txt
