# 48-B / 64-B / 128-B probes into the 4 GiB table beside the stream, cache policies: time, then
# FETCH_SIZE per dispatch (does any load policy fetch less than the L2's 128-B line?)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r6u}
mkdir -p $out
timeout -k 10 120 ./tools/mb_scatter 102 > $out/time.txt 2>&1 || exit 1
cat $out/time.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc -o run -- ./tools/mb_scatter 102 > $out/pmc.txt 2>&1 || exit 2
find $out/pmc -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} $out/fetch.csv
rm -rf $out/pmc
