#!/bin/bash
# tools/extra_round.sh TAG: config 3, host-staged (PCIe) and streaming measurements.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
[ -n "${SKIP_BENCH_EXTRA:-}" ] || timeout -k 10 300 python -u tools/bench_extra.py config3 > "$OUT/config3.json" 2> "$OUT/config3.err"
[ -n "${SKIP_BENCH_EXTRA:-}" ] || timeout -k 10 120 python -u tools/bench_extra.py pcie --seconds 8 > "$OUT/pcie.json" 2> "$OUT/pcie.err"
[ -n "${SKIP_BENCH_EXTRA:-}" ] || timeout -k 10 200 python -u tools/bench_extra.py stream --rate 1000000 --seconds 25 > "$OUT/stream.json" 2> "$OUT/stream.err"
cat "$OUT"/*.json || true
# the native runner on a generated 20M-event replay file (file read + host line split +
# pinned double buffers + H2D + kernel), the GPU stand-in for configs[0]'s local-mode job
D=/tmp/ysb_runner_data
rm -rf "$D" && mkdir -p "$D"
timeout -k 10 120 streaming-benchmarks_amd/bin/ysb_gen -d "$D" -n 20000000 --rate 100000 > /dev/null
printf 'ad_to_campaign_path: "%s/ad-to-campaign.csv"\nevents_path: "%s/kafka-json.txt"\nredis.host: "localhost"\n' "$D" "$D" > "$D/conf.yaml"
timeout -k 10 120 streaming-benchmarks_amd/bin/ysb_topology --confPath "$D/conf.yaml" --sink csv:"$D/w.csv" > "$OUT/runner.json"
tail -n 1 "$OUT/runner.json"
rm -rf "$D"
