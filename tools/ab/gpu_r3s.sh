#!/bin/bash
# Round 3, final tree: GPU tests, smoke, the default bench line, then configs[4] with 8
# shards on the one GPU for 40 s (the host side of an 8-GPU stream leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3s}; mkdir -p $O
bash tools/gpu_round.sh ${1:-r3s} tests smoke bench || exit 1
tail -2 $O/pytest_gpu.log
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value']/1e9, d['roofline']['frac'], d['check'])
print({k:(round(v.get('events_per_s',0)/1e9,3), v.get('hbm_frac'), v.get('error')) for k,v in d['extras'].items() if isinstance(v,dict)})
print(d['extras'].get('stream_sharded',{}).get('window_close_latency'), d['extras'].get('stream_sharded',{}).get('shards'))"
timeout -k 10 120 python3 -u tools/bench_extra.py stream_sharded --shards 8 --seconds 40 > $O/stream8.json 2> $O/stream8.err || { tail -20 $O/stream8.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/stream8.json')); print(d['shards'], d['window_close_latency'], d['exact_vs_generator_truth'])"
