set -o pipefail
mkdir -p gpurun_out/r5q
timeout -k 10 400 python -u -m pytest tests/test_gpu_raw.py tests/test_gpu_topology.py tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_ranks.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r5q/tests.log 2>&1 || { tail -30 gpurun_out/r5q/tests.log; exit 1; }
echo tests ok
timeout -k 10 300 python tools/h2d_diag.py --sdma --events 30000000 > gpurun_out/r5q/diag.json 2> gpurun_out/r5q/diag.err || exit 1
echo diag ok
timeout -k 10 300 python tools/bench_stream.py --seconds 6 > gpurun_out/r5q/stream.json 2> gpurun_out/r5q/stream.err || { tail -20 gpurun_out/r5q/stream.err; exit 1; }
echo stream ok
timeout -k 10 300 python -c "
import argparse, json, sys; sys.argv=['bench.py']; import bench
a = bench.parse_args([])
print(json.dumps(bench.extra_alternating(a, 0)))" > gpurun_out/r5q/alt.json 2> gpurun_out/r5q/alt.err
echo "alt rc=$?"
