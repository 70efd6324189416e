# SQ LDS counters of the .tbl stage-1 variants (production, '|' bitmap, ds_read_b64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in base bm r64s; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  OUT=gpurun_out/r3l/$v CMD="tools/extra_one.py tbl --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
done
