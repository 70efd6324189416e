set -o pipefail
mkdir -p gpurun_out/r5k
cat > /tmp/alt.py <<'PY'
import json, os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tools"), os.path.join(os.getcwd(), "streaming-benchmarks_amd")]
import bench_dropin
out = []
for k in range(5):
    for raw in (False, True):
        r = bench_dropin.host_staged(0, 20_000_000, raw=raw)
        out.append(("raw" if raw else "offsets", r["h2d_GBs"]))
print(json.dumps(out))
PY
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r5k/tr -o tr -- python3 /tmp/alt.py > gpurun_out/r5k/alt.json 2> gpurun_out/r5k/alt.err
echo "rc=$?"
