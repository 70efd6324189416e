set -o pipefail
mkdir -p gpurun_out/r5g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r5g/tr -o tr -- python3 tools/h2d_diag.py --events 20000000 > gpurun_out/r5g/diag.json 2> gpurun_out/r5g/diag.err
echo "rc=$?"
ls -R gpurun_out/r5g | head -30
