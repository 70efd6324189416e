set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5mixsq; mkdir -p $O
export YSB_LIB_VARIANT=mixnd
OUT=$O/sq_mixnd CMD="tools/extra_one.py reorder_flat_fixed --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
echo done
