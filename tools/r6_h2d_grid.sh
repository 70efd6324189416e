# Does the copy kernel's request load starve the HBM work beside it?  Copy-kernel grid
# (YSB_H2D_GRID workgroups of 256 threads) x split placement, streaming runner, 220M asked.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r6r}
mkdir -p $out
R=streaming-benchmarks_amd/bin/ysb_topology
for v in "256 0 mapped-raw" "64 0 mapped-raw" "64 1 mapped-raw" "32 1 mapped-raw" "128 1 mapped-raw" "256 0 mapped" "64 0 mapped" "32 0 mapped"; do
  set -- $v
  YSB_H2D_GRID=$1 YSB_SPLIT_STREAM=$2 timeout -k 10 200 $R --stream --sink none --seconds 8 --event-rate 6285714 --speedup 35 --replay $3 > $out/g$1_s$2_$3.json 2> $out/g$1_s$2_$3.err || exit 2
  python -c "import json; r=json.loads(open('$out/g$1_s$2_$3.json').read().strip().splitlines()[-1]); print('grid', $1, 'split', $2, '$3', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'])"
done
