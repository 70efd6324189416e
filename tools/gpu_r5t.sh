# round 5: the raw split behind the copy kernel on the copy stream -- raw / topology / stream
# GPU tests, then the runner (copy kernel vs DMA engine) and the native stream
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_topology.py tests/test_gpu_stream.py > $O/tests.log 2>&1 || tail -30 $O/tests.log
tail -1 $O/tests.log
W=/tmp/ysb_r5t_replay
for r in 1 2; do
  for m in kernel sdma; do
    F=""; [ $m = sdma ] && F="--h2d-sdma"
    timeout -k 10 200 python3 tools/bench_dropin.py runner --workdir $W $F > $O/runner_${m}_$r.json 2> $O/runner_${m}_$r.err || { tail -5 $O/runner_${m}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/runner_${m}_$r.json'));print('$m', d['stream_events_per_s']/1e6, d['stream_GBs'], d['copy_GBs'], d['copy_busy_frac'], d['fill_s'], d['slot_wait_s'], d['stream_seconds'], d['check']['truth_mismatched_cells'])"
  done
done
timeout -k 10 200 python3 tools/bench_dropin.py staged --raw > $O/staged_raw.json 2> $O/staged_raw.err || exit 1
python3 -c "import json;d=json.load(open('$O/staged_raw.json'));print('staged raw', d['events_per_s']/1e6, d['h2d_GBs'], d['copy_busy_frac'], d['check']['truth_mismatched_cells'])"
timeout -k 10 300 python3 tools/bench_stream.py --seconds 8 --speedup 40 > $O/stream40.json 2> $O/stream40.err || { tail -5 $O/stream40.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/stream40.json'));print('stream', d['events_per_s']/1e6, d['target_events_per_s']/1e6, d['copy_GBs'], d['copy_busy_frac'], d['max_behind_ms'], d['get_stats']['p50_ms'], d['get_stats']['p99_ms'], d['exact_vs_generator_truth'])"
