set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/flatprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/flatprof/p -o run -- python3 $R/tools/bench_extra.py general --shape reorder --steps 5 > $R/gpurun_out/flatprof/out.json 2> $R/gpurun_out/flatprof/err.log
