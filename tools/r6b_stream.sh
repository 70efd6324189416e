set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 300 python -u -m pytest tests/test_gpu_topology.py tests/test_gpu_mapped.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6b/tests.log 2>&1 || exit 1
for mode in mapped copy; do
  timeout -k 10 200 python tools/bench_stream.py --seconds 12 --event-rate 5857142 --speedup 35 --replay $mode > gpurun_out/r6b/stream_$mode.json 2> gpurun_out/r6b/stream_$mode.err || exit 2
done
timeout -k 10 200 python tools/bench_stream.py --seconds 12 --event-rate 2928571 --speedup 35 --shards 2 --replay mapped > gpurun_out/r6b/stream_mapped_2sh.json 2> gpurun_out/r6b/stream_mapped_2sh.err || exit 3
echo done
