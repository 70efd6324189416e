# config 3 after the packed 64-B buckets + u8 delta: tests, two timed runs, trace, PMC traffic
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_records.py tests/test_gpu_ranks.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do timeout -k 10 300 python -u tools/extra_one.py config3 > $O/c3_$i.json 2> $O/c3_$i.err || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/extra_one.py config3 --extra-steps 5 --warmup 2 > $O/trace.json 2> $O/trace.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 tools/extra_one.py config3 --extra-steps 2 --warmup 1 > $O/pmc_fetch.json 2>$O/pmc_fetch.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 tools/extra_one.py config3 --extra-steps 2 --warmup 1 > $O/pmc_write.json 2>$O/pmc_write.err || exit 1
for k in scan_kernel rec_partition rec_count; do echo "== $k"; python3 tools/pmc_summary.py $O $k | tail -4; done
python3 -c "
import json
for i in (1,2):
    d=json.load(open('$O/c3_%d.json'%i)); print(d['events_per_s']/1e9, d['hbm_frac'], d['avg_launch_ms'], d['avg_path_ms'], d['check'])
"
