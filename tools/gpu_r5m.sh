# DPM hypothesis: after an idle period the SOC / fabric clocks are low and a copy-bound leg
# (one short kernel per 256 MB copy) does not raise them.  Sample the DPM levels during legs.
set -o pipefail
mkdir -p gpurun_out/r5m
dev=$(ls -d /sys/class/drm/card*/device | head -1)
for f in pp_dpm_sclk pp_dpm_mclk pp_dpm_fclk pp_dpm_socclk pp_dpm_dcefclk pp_dpm_pcie power_dpm_force_performance_level gpu_busy_percent current_link_speed current_link_width; do echo "== $f"; cat $dev/$f 2>&1; done > gpurun_out/r5m/dpm_idle.txt
( for i in $(seq 1 400); do echo "t=$i $(grep '\*' $dev/pp_dpm_socclk | tr -d '\n') | $(grep '\*' $dev/pp_dpm_fclk | tr -d '\n') | $(grep '\*' $dev/pp_dpm_mclk | tr -d '\n') | busy $(cat $dev/gpu_busy_percent)"; sleep 0.1; done > gpurun_out/r5m/dpm_series.txt ) &
SAMPLER=$!
sleep 3
timeout -k 10 200 python tools/h2d_diag.py --events 30000000 > gpurun_out/r5m/diag.json 2> gpurun_out/r5m/diag.err
rc=$?
kill $SAMPLER 2>/dev/null
echo rc=$rc
