# round-3 evidence: headline trace + PMC traffic + full bench line (final_profile.sh), config-3 trace + PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3m; mkdir -p $O
bash tools/final_profile.sh r3m || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3trace -o run -- python3 tools/extra_one.py config3 > $O/c3trace.json 2> $O/c3trace.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3pmc/pmc_fetch -o run -- python3 tools/extra_one.py config3 --extra-steps 2 --warmup 1 > $O/c3pmc_fetch.json 2>$O/c3pmc_fetch.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3pmc/pmc_write -o run -- python3 tools/extra_one.py config3 --extra-steps 2 --warmup 1 > $O/c3pmc_write.json 2>$O/c3pmc_write.err || exit 1
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value']/1e9, d['roofline']); print({k:(v.get('events_per_s',0)/1e9, v.get('hbm_frac'), v.get('error')) for k,v in d['extras'].items() if isinstance(v,dict)}); print(d['extras'].get('stream_sharded',{}).get('window_close_latency'))"
