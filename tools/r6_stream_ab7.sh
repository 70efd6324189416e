# split on its own stream now that the copy queue skips satisfied barriers, 1 GPU (+ a trace of it)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r6j}
mkdir -p $out
R=streaming-benchmarks_amd/bin/ysb_topology
for s in 1 0 1 0; do
  YSB_SPLIT_STREAM=$s timeout -k 10 200 $R --stream --sink none --seconds 10 --event-rate 6285714 --speedup 35 > $out/s$s.json 2> $out/s$s.err || exit 2
  python -c "import json; r=json.loads(open('$out/s$s.json').read().strip().splitlines()[-1]); print('split', $s, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'])"
done
YSB_SPLIT_STREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- $R --stream --sink none --seconds 3 --event-rate 6285714 --speedup 35 > $out/tr.json 2> $out/tr.err || exit 3
find $out/trace -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $out/kernel_trace_s1.csv
rm -rf $out/trace
