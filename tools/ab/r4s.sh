#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 120 python3 tools/h2d_probe.py > $O/probe.json 2> $O/probe.err || exit 1
cat $O/probe.json
for mb in 64 256; do
  timeout -k 10 200 python3 tools/bench_dropin.py staged --slot-mb $mb --events 50000000 > $O/staged_$mb.json 2> $O/staged_$mb.err || exit 1
  python3 -c "import json;d=json.load(open('$O/staged_$mb.json'));print($mb, {k:d[k] for k in ('events_per_s','h2d_GBs','h2d_ms_per_batch','copy_busy_frac')})"
done
