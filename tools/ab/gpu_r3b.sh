# A/B: layout sampling of device batches (default) vs YSB_F_LAYOUT_FIXED on the headline,
# then the extras (no stream) on the new tree.
set -o pipefail
mkdir -p gpurun_out/r3b
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu --no-check > gpurun_out/r3b/a$i.json 2> gpurun_out/r3b/a$i.err || exit 1
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu --no-check --layout-fixed > gpurun_out/r3b/b$i.json 2> gpurun_out/r3b/b$i.err || exit 1
done
timeout -k 10 900 python -u bench.py --no-cpu --stream-seconds 0 > gpurun_out/r3b/full.json 2> gpurun_out/r3b/full.err || exit 1
python - <<'PY'
import json
for n in ("a1","b1","a2","b2"):
    d=json.load(open("gpurun_out/r3b/%s.json"%n)); print(n, d["value"]/1e9, d["roofline"]["avg_launch_ms"], d["roofline"]["kernel"])
d=json.load(open("gpurun_out/r3b/full.json"))
print("headline", d["value"]/1e9, d["check"])
for k,v in d["extras"].items():
    print(k, v.get("events_per_s",0)/1e9, v.get("hbm_frac"), v.get("kernel"), v.get("check",{}).get("truth_mismatched_cells"), v.get("error"))
PY
