# Copy-kernel grid / split placement on the drop-in legs (host_staged: offsets, raw, DMA
# engine; native_runner: the file replay) and the stream, same box, two alternations.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r6s}
mkdir -p $out
R=streaming-benchmarks_amd/bin/ysb_topology
for rep in 1 2; do
for v in "0 0" "32 1" "16 1" "32 0"; do
  set -- $v
  tag=g$1_s$2_r$rep
  YSB_H2D_GRID=$1 YSB_SPLIT_STREAM=$2 timeout -k 10 300 python tools/extra_one.py host_staged --dropin-events 50000000 > $out/hs_$tag.json 2> $out/hs_$tag.err || exit 2
  YSB_H2D_GRID=$1 YSB_SPLIT_STREAM=$2 timeout -k 10 300 python tools/extra_one.py native_runner --runner-file-events 10000000 --runner-repeat 4 > $out/nr_$tag.json 2> $out/nr_$tag.err || exit 3
  YSB_H2D_GRID=$1 YSB_SPLIT_STREAM=$2 timeout -k 10 200 $R --stream --sink none --seconds 6 --event-rate 6285714 --speedup 35 --replay mapped-raw > $out/st_$tag.json 2> $out/st_$tag.err || exit 4
  python - <<PY
import json
h=json.loads(open('$out/hs_$tag.json').read().strip().splitlines()[-1]); n=json.loads(open('$out/nr_$tag.json').read().strip().splitlines()[-1]); s=json.loads(open('$out/st_$tag.json').read().strip().splitlines()[-1])
print('$tag', 'staged off/raw/dma %.1f %.1f %.1f' % (h['offsets']['events_per_s']/1e6, h['raw']['events_per_s']/1e6, h['offsets_dma_engine']['events_per_s']/1e6), 'runner %.1f %.1f' % (n['gpu_split']['stream_events_per_s']/1e6, n['gpu_split_dma_engine']['stream_events_per_s']/1e6), 'stream-raw %.1f' % (s['events_per_s']/1e6))
PY
done
done
