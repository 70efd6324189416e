set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_group_host.py -x -v -k pipelined --timeout 300 --timeout-method thread > $O/group.log 2>&1 || { tail -40 $O/group.log; exit 1; }
tail -4 $O/group.log
timeout -k 10 300 python -u tools/exchange_cost.py > $O/xcost.json 2> $O/xcost.err || { tail -20 $O/xcost.err; exit 1; }
cat $O/xcost.json
