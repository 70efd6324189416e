#!/bin/bash
# Round evidence run (GPU box, tools/round_final.sh TAG b): configs[2] trace + PMC traffic,
# the raw drop-in path's kernel trace (the GPU line split beside the scan), the mixed-layout
# leg's trace, the native streaming mode's trace (copy kernel, scan, flush compaction).
#   tools/round_profile.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-rf}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3trace -o run -- python3 tools/extra_one.py config3 > $O/c3trace.json 2> $O/c3trace.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3pmc/pmc_fetch -o run -- python3 tools/extra_one.py config3 --extra-steps 2 --warmup 1 > $O/c3pmc_fetch.json 2>$O/c3pmc_fetch.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3pmc/pmc_write -o run -- python3 tools/extra_one.py config3 --extra-steps 2 --warmup 1 > $O/c3pmc_write.json 2>$O/c3pmc_write.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rawtrace -o run -- python3 tools/bench_dropin.py staged --raw --events 20000000 > $O/rawtrace.json 2> $O/rawtrace.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mixtrace -o run -- python3 tools/extra_one.py mixed_flat_fixed > $O/mixtrace.json 2> $O/mixtrace.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/streamtrace -o run -- streaming-benchmarks_amd/bin/ysb_topology --stream --sink none --seconds 4 --speedup 35 --event-rate 5771428 > $O/streamtrace.json 2> $O/streamtrace.err || exit 1
echo "round profile done"
