# round 5: the native runner's H2D by the copy kernel vs the DMA engine (same replay file,
# alternated), then the flat tier's one-round-trip span A/B (tools/ab_flat.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s; mkdir -p $O
W=/tmp/ysb_r5s_replay
for r in 1 2; do
  for m in kernel sdma; do
    F=""; [ $m = sdma ] && F="--h2d-sdma"
    timeout -k 10 200 python3 tools/bench_dropin.py runner --workdir $W $F > $O/runner_${m}_$r.json 2> $O/runner_${m}_$r.err || { tail -5 $O/runner_${m}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/runner_${m}_$r.json'));print('$m', d['stream_events_per_s']/1e6, d['stream_GBs'], d['copy_GBs'], d['copy_busy_frac'], d['fill_s'], d['slot_wait_s'], d['stream_seconds'], d['check']['truth_mismatched_cells'])"
  done
done
bash tools/ab_flat.sh r5s base span
