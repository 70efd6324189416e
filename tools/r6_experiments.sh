#!/bin/bash
# Round 6's GPU experiments, one function each (the gpurun_out tags AB_LOG.md and DESIGN.md cite):
#   bash tools/r6_experiments.sh NAME [TAG]     e.g. bash tools/r6_experiments.sh copy_grid r6r
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"

stream_first() {  # default tag r6b
mkdir -p gpurun_out/r6b
timeout -k 10 300 python -u -m pytest tests/test_gpu_topology.py tests/test_gpu_mapped.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6b/tests.log 2>&1 || exit 1
for mode in mapped copy; do
  timeout -k 10 200 python tools/bench_stream.py --seconds 12 --event-rate 5857142 --speedup 35 --replay $mode > gpurun_out/r6b/stream_$mode.json 2> gpurun_out/r6b/stream_$mode.err || exit 2
done
timeout -k 10 200 python tools/bench_stream.py --seconds 12 --event-rate 2928571 --speedup 35 --shards 2 --replay mapped > gpurun_out/r6b/stream_mapped_2sh.json 2> gpurun_out/r6b/stream_mapped_2sh.err || exit 3
echo done
}

# A/B of the streaming feed's copy stream (diagnostic knobs YSB_SPLIT_STREAM / YSB_H2D_WG), 1 GPU
split_grid_ab() {  # default tag r6c
out=gpurun_out/${TAG:-r6c}
mkdir -p $out
for v in "0 1" "1 1" "0 2" "1 2" "0 1"; do
  set -- $v
  YSB_SPLIT_STREAM=$1 YSB_H2D_WG=$2 timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 > $out/s$1_w$2.json 2> $out/s$1_w$2.err || exit 2
  python -c "import json; r=json.load(open('$out/s$1_w$2.json')); print('split', $1, 'wg', $2, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['exact_vs_generator_truth'])"
done
timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 --batch-ms 200 > $out/b200.json 2> $out/b200.err || exit 3
python -c "import json; r=json.load(open('$out/b200.json')); print('batch 200', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['exact_vs_generator_truth'])"
}

# A/B of the streaming feed after the copy queue's barrier skip, 1 GPU
barrier_skip() {  # default tag r6d
out=gpurun_out/${TAG:-r6d}
mkdir -p $out
for v in "100 mapped" "200 mapped" "100 copy"; do
  set -- $v
  timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 --batch-ms $1 --replay $2 > $out/b$1_$2.json 2> $out/b$1_$2.err || exit 2
  python -c "import json; r=json.load(open('$out/b$1_$2.json')); print('batch', $1, '$2', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['exact_vs_generator_truth'])"
done
}

# same-box: host_staged raw vs the stream at several batch sizes / flush periods, 1 GPU
vs_host_staged() {  # default tag r6e
out=gpurun_out/${TAG:-r6e}
mkdir -p $out
timeout -k 10 200 python -c "
import sys, json; sys.path[:0] = ['tools', 'streaming-benchmarks_amd']
import bench_dropin
r = bench_dropin.host_staged(0, 100_000_000, raw=True)
print(json.dumps(r))" > $out/host_staged.json 2> $out/host_staged.err || exit 1
python -c "import json; r=json.load(open('$out/host_staged.json')); print('host_staged raw', round(r['events_per_s']/1e6,1), r['h2d_GBs'], r['copy_busy_frac'], r['h2d_ms_per_batch'])"
for v in "100 1000" "300 1000" "100 100000"; do
  set -- $v
  timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 --batch-ms $1 --flush-ms $2 > $out/b$1_f$2.json 2> $out/b$1_f$2.err || exit 2
  python -c "import json; r=json.load(open('$out/b$1_f$2.json')); print('batch', $1, 'flush', $2, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'], r['exact_vs_generator_truth'])"
done
}

# stream copy rate vs the replay cycle's size (IOMMU / TLB reach?), 1 GPU; THP state
cycle_size() {  # default tag r6f
out=gpurun_out/${TAG:-r6f}
mkdir -p $out
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $out/thp.txt 2>&1
ls /sys/kernel/iommu_groups 2>/dev/null | wc -l >> $out/thp.txt
cat /sys/class/iommu/*/devices 2>/dev/null | head -2 >> $out/thp.txt
dmesg 2>/dev/null | grep -i -m3 iommu >> $out/thp.txt
for v in "6285714 35 100" "1257143 175 500" "314286 700 2000"; do
  set -- $v
  timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate $1 --speedup $2 --batch-ms $3 > $out/r$1.json 2> $out/r$1.err || exit 2
  python -c "import json; r=json.load(open('$out/r$1.json')); print('rate', $1, 'speedup', $2, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'], r['per_shard'][0]['replay_GB'], r['exact_vs_generator_truth'])"
done
cat $out/thp.txt
}

# stream rate with / without the copy-timing markers, split on the copy stream / its own, 1 GPU
timing_markers() {  # default tag r6g
out=gpurun_out/${TAG:-r6g}
mkdir -p $out
R=streaming-benchmarks_amd/bin/ysb_topology
for v in "0 t" "0 n" "1 n" "0 t"; do
  set -- $v
  extra=""; [ "$2" = n ] && extra="--no-timing"
  YSB_SPLIT_STREAM=$1 timeout -k 10 200 $R --stream --sink none --seconds 10 --event-rate 6285714 --speedup 35 $extra > $out/s$1_$2.json 2> $out/s$1_$2.err || exit 2
  python -c "import json; r=json.loads(open('$out/s$1_$2.json').read().strip().splitlines()[-1]); print('split', $1, '$2', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'])"
done
}

# stream rate with the copy kernel at raised wave priority, 1 GPU
copy_prio() {  # default tag r6h
out=gpurun_out/${TAG:-r6h}
mkdir -p $out
R=streaming-benchmarks_amd/bin/ysb_topology
for p in 0 1 0 1; do
  YSB_H2D_PRIO=$p timeout -k 10 200 $R --stream --sink none --seconds 10 --event-rate 6285714 --speedup 35 > $out/p$p.json 2> $out/p$p.err || exit 2
  python -c "import json; r=json.loads(open('$out/p$p.json').read().strip().splitlines()[-1]); print('prio', $p, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'])"
done
}

# kernel trace of the streaming runner (gaps between the slot copies), 1 GPU
trace() {  # default tag r6i
out=gpurun_out/${TAG:-r6i}
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- streaming-benchmarks_amd/bin/ysb_topology --stream --sink none --seconds 3 --event-rate 6285714 --speedup 35 > $out/run.json 2> $out/run.err || exit 2
find $out/trace -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $out/kernel_trace.csv
ls -la $out
}

# split on its own stream now that the copy queue skips satisfied barriers, 1 GPU (+ a trace of it)
split_own_stream() {  # default tag r6j
out=gpurun_out/${TAG:-r6j}
mkdir -p $out
R=streaming-benchmarks_amd/bin/ysb_topology
for s in 1 0 1 0; do
  YSB_SPLIT_STREAM=$s timeout -k 10 200 $R --stream --sink none --seconds 10 --event-rate 6285714 --speedup 35 > $out/s$s.json 2> $out/s$s.err || exit 2
  python -c "import json; r=json.loads(open('$out/s$s.json').read().strip().splitlines()[-1]); print('split', $s, round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'])"
done
YSB_SPLIT_STREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- $R --stream --sink none --seconds 3 --event-rate 6285714 --speedup 35 > $out/tr.json 2> $out/tr.err || exit 3
find $out/trace -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $out/kernel_trace_s1.csv
rm -rf $out/trace
}

# mapped tests + the three replay modes, 1 GPU
replay_modes() {  # default tag r6k
out=gpurun_out/${TAG:-r6k}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mapped.py tests/test_gpu_topology.py -x -v --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
grep -c PASSED $out/tests.log
for m in mapped mapped-raw mapped copy; do
  timeout -k 10 200 python tools/bench_stream.py --seconds 10 --event-rate 6285714 --speedup 35 --replay $m > $out/$m.json 2> $out/$m.err || exit 2
  python -c "import json; r=json.load(open('$out/$m.json')); print('$m', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'], r['batches'], r['exact_vs_generator_truth'], r['get_stats']['p50_ms'], r['get_stats']['p99_ms'])"
done
}

# configs[2]: do 128-B probes into a table that fits the 256 MiB Infinity Cache leave HBM beside
# the scan's nontemporal 25.8 GB stream?  tools/mb_scatter 13: time per table size, then
# FETCH_SIZE (x2, gfx950) and WRITE_SIZE per dispatch in passes of their own.
icache() {  # default tag r6l
out=gpurun_out/${TAG:-r6l}
mkdir -p $out
timeout -k 10 120 ./tools/mb_scatter 13 > $out/mb13_time.txt 2>&1 || exit 1
cat $out/mb13_time.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $out/pmc_$c -o run -- ./tools/mb_scatter 13 > $out/mb13_$c.txt 2>&1 || exit 2
  find $out/pmc_$c -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} $out/mb13_$c.csv
  rm -rf $out/pmc_$c
done
}

# The structural index's classification alone (YSB_DIAG_FLAT_IDX) against the flat tier's whole
# parse (no probe, no count) and Phase A alone, layout 2 forced, mixed and reordered producers.
flat_index() {  # default tag r6m
out=gpurun_out/${TAG:-r6m}
mkdir -p $out
for leg in mixed_flat_fixed reorder_flat_fixed; do
  for v in none fidx flatnj diag; do
    vv=$v; [ $v = none ] && vv=""
    YSB_LIB_VARIANT=$vv timeout -k 10 200 python tools/extra_one.py $leg --extra-steps 10 --warmup 3 > $out/${leg}_$v.json 2> $out/${leg}_$v.err || { tail -3 $out/${leg}_$v.err; exit 2; }
    python -c "import json; r=json.loads(open('$out/${leg}_$v.json').read().strip().splitlines()[-1]); print('$leg', '$v', r['avg_launch_ms'], r['events_per_s']/1e9)"
  done
done
for v in none fidx; do
  vv=$v; [ $v = none ] && vv=""
  YSB_LIB_VARIANT=$vv timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d $out/pmc_$v -o run -- python3 tools/extra_one.py mixed_flat_fixed --extra-steps 2 --warmup 1 > $out/pmc_$v.json 2> $out/pmc_$v.err || exit 3
  find $out/pmc_$v -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} $out/sq_$v.csv
  rm -rf $out/pmc_$v
done
}

# Does the copy kernel's request load starve the HBM work beside it?  Copy-kernel grid
# (YSB_H2D_GRID workgroups of 256 threads) x split placement, streaming runner, 220M asked.
copy_grid() {  # default tag r6r
out=gpurun_out/${TAG:-r6r}
mkdir -p $out
R=streaming-benchmarks_amd/bin/ysb_topology
for v in "256 0 mapped-raw" "64 0 mapped-raw" "64 1 mapped-raw" "32 1 mapped-raw" "128 1 mapped-raw" "256 0 mapped" "64 0 mapped" "32 0 mapped"; do
  set -- $v
  YSB_H2D_GRID=$1 YSB_SPLIT_STREAM=$2 timeout -k 10 200 $R --stream --sink none --seconds 8 --event-rate 6285714 --speedup 35 --replay $3 > $out/g$1_s$2_$3.json 2> $out/g$1_s$2_$3.err || exit 2
  python -c "import json; r=json.loads(open('$out/g$1_s$2_$3.json').read().strip().splitlines()[-1]); print('grid', $1, 'split', $2, '$3', round(r['events_per_s']/1e6,1), r['copy_GBs'], r['copy_busy_frac'])"
done
}

# Copy-kernel grid / split placement on the drop-in legs (host_staged: offsets, raw, DMA
# engine; native_runner: the file replay) and the stream, same box, two alternations.
copy_grid_dropin() {  # default tag r6s
out=gpurun_out/${TAG:-r6s}
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
}

# the new copy-grid / split defaults: raw / mapped / topology tests, then the legs once
copy_grid_confirm() {  # default tag r6t
out=gpurun_out/${TAG:-r6t}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_raw.py tests/test_gpu_mapped.py tests/test_gpu_topology.py tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python tools/extra_one.py host_staged > $out/hs.json 2> $out/hs.err || exit 2
timeout -k 10 300 python tools/extra_one.py native_runner > $out/nr.json 2> $out/nr.err || exit 3
timeout -k 10 200 python tools/bench_stream.py --seconds 8 --event-rate 6285714 --speedup 35 --replay mapped-raw > $out/st_raw.json 2> $out/st_raw.err || exit 4
python - <<PY
import json
h=json.loads(open('$out/hs.json').read().strip().splitlines()[-1]); n=json.loads(open('$out/nr.json').read().strip().splitlines()[-1]); s=json.load(open('$out/st_raw.json'))
print('staged off/raw/dma %.1f %.1f %.1f' % (h['offsets']['events_per_s']/1e6, h['raw']['events_per_s']/1e6, h['offsets_dma_engine']['events_per_s']/1e6), 'h2d GB/s', h['raw']['h2d_GBs'], 'runner %.1f host %.1f dma %.1f' % (n['gpu_split']['stream_events_per_s']/1e6, n['host_split']['stream_events_per_s']/1e6, n['gpu_split_dma_engine']['stream_events_per_s']/1e6), 'stream-raw %.1f exact %s' % (s['events_per_s']/1e6, s['exact_vs_generator_truth']))
PY
}

# 48-B / 64-B / 128-B probes into the 4 GiB table beside the stream, cache policies: time, then
# FETCH_SIZE per dispatch (does any load policy fetch less than the L2's 128-B line?)
probe_policy() {  # default tag r6u
out=gpurun_out/${TAG:-r6u}
mkdir -p $out
timeout -k 10 120 ./tools/mb_scatter 102 > $out/time.txt 2>&1 || exit 1
cat $out/time.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc -o run -- ./tools/mb_scatter 102 > $out/pmc.txt 2>&1 || exit 2
find $out/pmc -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} $out/fetch.csv
rm -rf $out/pmc
}

name=$1; TAG=${2:-}
declare -F "$name" > /dev/null || { echo "unknown experiment: $name"; exit 2; }
"$name"
