# kernel trace of the streaming runner (gaps between the slot copies), 1 GPU
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r6i}
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- streaming-benchmarks_amd/bin/ysb_topology --stream --sink none --seconds 3 --event-rate 6285714 --speedup 35 > $out/run.json 2> $out/run.err || exit 2
find $out/trace -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $out/kernel_trace.csv
ls -la $out
