set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "alternating or sticky or carries or device_count or follows_a_producer" > gpurun_out/r5a/new_tests.log 2>&1
echo "new tests rc=$?"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5a/tests.log 2>&1 || { echo "suite rc=$?"; tail -30 gpurun_out/r5a/tests.log; exit 1; }
timeout -k 10 180 python tools/h2d_probe.py --after-load > gpurun_out/r5a/probe.json 2> gpurun_out/r5a/probe.err && \
timeout -k 10 400 python tools/h2d_diag.py > gpurun_out/r5a/diag.json 2> gpurun_out/r5a/diag.err
echo "diag rc=$?"
