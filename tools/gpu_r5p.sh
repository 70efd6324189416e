set -o pipefail
mkdir -p gpurun_out/r5p
timeout -k 10 400 python -u -m pytest tests/test_gpu_raw.py tests/test_gpu_topology.py tests/test_gpu_stream.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r5p/tests.log 2>&1 || { tail -30 gpurun_out/r5p/tests.log; exit 1; }
timeout -k 10 300 python tools/h2d_diag.py --sdma --events 30000000 > gpurun_out/r5p/diag.json 2> gpurun_out/r5p/diag.err || exit 1
timeout -k 10 300 python tools/bench_stream.py --seconds 6 > gpurun_out/r5p/stream.json 2> gpurun_out/r5p/stream.err
echo "stream rc=$?"
