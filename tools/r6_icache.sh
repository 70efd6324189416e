# configs[2]: do 128-B probes into a table that fits the 256 MiB Infinity Cache leave HBM beside
# the scan's nontemporal 25.8 GB stream?  tools/mb_scatter 13: time per table size, then
# FETCH_SIZE (x2, gfx950) and WRITE_SIZE per dispatch in passes of their own.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r6l}
mkdir -p $out
timeout -k 10 120 ./tools/mb_scatter 13 > $out/mb13_time.txt 2>&1 || exit 1
cat $out/mb13_time.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $out/pmc_$c -o run -- ./tools/mb_scatter 13 > $out/mb13_$c.txt 2>&1 || exit 2
  find $out/pmc_$c -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} $out/mb13_$c.csv
  rm -rf $out/pmc_$c
done
