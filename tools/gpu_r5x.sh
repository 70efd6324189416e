# round 5 A/B, repeated: the raw split on the copy stream (0) vs the compute stream (1) (YSB_AB_SPLIT, a temporary switch, removed after it), the
# native runner with the copy kernel, 4 alternations; the DMA engine as a reference
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5x; mkdir -p $O
W=/tmp/ysb_r5x_replay
for r in 1 2 3 4; do
  for m in 0 1; do
    F=""; E=$m; [ $m = sdma ] && { F="--h2d-sdma"; E=0; }
    YSB_AB_SPLIT=$E timeout -k 10 200 python3 tools/bench_dropin.py runner --workdir $W $F > $O/runner_${m}_$r.json 2> $O/runner_${m}_$r.err || { tail -5 $O/runner_${m}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/runner_${m}_$r.json'));print('$m', round(d['stream_events_per_s']/1e6,1), d['copy_GBs'], d['copy_busy_frac'], 'fill', d['fill_s'], 'stream_s', d['stream_seconds'], 'non-fill', round(d['stream_seconds']-d['fill_s'],3), d['check']['truth_mismatched_cells'])"
  done
done
