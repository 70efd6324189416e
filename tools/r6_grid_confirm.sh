# the new copy-grid / split defaults: raw / mapped / topology tests, then the legs once
set -o pipefail
out=gpurun_out/${1:-r6t}
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
