set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3a/tests.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/r3a/tests.log
tail -5 gpurun_out/r3a/tests.log
