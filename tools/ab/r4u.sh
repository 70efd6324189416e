#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 120 python3 tools/h2d_probe.py > $O/probe.json 2> $O/probe.err || exit 1
cat $O/probe.json
for ev in 50000000 100000000; do
  timeout -k 10 200 python3 tools/bench_dropin.py staged --events $ev > $O/staged_$ev.json 2> $O/staged_$ev.err || exit 1
  python3 -c "import json;d=json.load(open('$O/staged_$ev.json'));print($ev, {k:d[k] for k in ('events_per_s','h2d_GBs','h2d_ms_per_batch','copy_busy_frac','batches')})"
done
timeout -k 10 300 python3 tools/bench_dropin.py runner > $O/runner.json 2> $O/runner.err || exit 1
python3 -c "import json;d=json.load(open('$O/runner.json'));print({k:d.get(k) for k in ('events_per_s','stream_events_per_s','stream_GBs','batches','seconds','stream_seconds')})"
