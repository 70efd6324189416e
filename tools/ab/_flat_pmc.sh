set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export OUT=gpurun_out/flatpmc
export BENCH="tools/bench_extra.py general --shape reorder --steps 2"
bash tools/pmc_sq.sh
export OUT=gpurun_out/flatpmc_gen
export BENCH="tools/bench_extra.py general --shape generator --steps 2"
bash tools/pmc_sq.sh
