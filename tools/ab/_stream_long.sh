set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/streamlong; mkdir -p $OUT
for n in 1 2 4 8; do
  timeout -k 10 280 python -u tools/bench_extra.py stream_sharded --shards $n --rate 2000000 --seconds 200 --batch-ms 20 > $OUT/n$n.json 2> $OUT/n$n.err
  python3 -c "import json;d=json.load(open('$OUT/n$n.json'));print($n, d['window_close_latency'], d['exact_vs_batch_path'], d['events'])"
done
