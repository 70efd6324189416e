# H2D gap diagnosis: each precondition of bench.py's headline phase alone, in a fresh
# process, then the host-staged offsets / raw legs; then a memory-copy trace of the full
# sequence.
set -o pipefail
mkdir -p gpurun_out/r5b
for pre in none torch segments pageable oracle; do
  timeout -k 10 150 python tools/h2d_diag.py --pre $pre --events 30000000 > gpurun_out/r5b/pre_$pre.json 2> gpurun_out/r5b/pre_$pre.err || { echo "pre $pre failed rc=$?"; exit 1; }
  echo "pre $pre done"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace --stats -d gpurun_out/r5b/mc -o mc -- python3 tools/h2d_diag.py --events 20000000 > gpurun_out/r5b/trace_diag.json 2> gpurun_out/r5b/trace_diag.err
echo "trace rc=$?"
