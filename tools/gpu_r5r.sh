set -o pipefail
mkdir -p gpurun_out/r5r
timeout -k 10 300 python -u -m pytest tests/test_gpu_ranks.py tests/test_gpu_stream.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r5r/tests.log 2>&1 || { tail -30 gpurun_out/r5r/tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python tools/bench_stream.py --seconds 12 > gpurun_out/r5r/stream.json 2> gpurun_out/r5r/stream.err || { tail -20 gpurun_out/r5r/stream.err; exit 1; }
echo stream ok
