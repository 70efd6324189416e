set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export OUT=gpurun_out/c3pmc2
export BENCH="tools/bench_extra.py config3 --steps 2 --warmup 1"
bash tools/profile.sh pmc fetch FETCH_SIZE
bash tools/profile.sh pmc write WRITE_SIZE
