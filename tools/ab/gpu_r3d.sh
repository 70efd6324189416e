# SQ counters: headline kernel (final-tree refresh), flat-first on reordered keys, .tbl
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r3d/head CMD="bench.py --steps 2 --warmup 1 --no-cpu --no-check --no-extras" bash tools/sq_passes.sh || exit 1
OUT=gpurun_out/r3d/flat CMD="tools/extra_one.py reorder --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
OUT=gpurun_out/r3d/tbl CMD="tools/extra_one.py tbl --extra-steps 2 --warmup 1" bash tools/sq_passes.sh || exit 1
for d in head flat tbl; do echo "== $d"; python3 tools/pmc_summary.py gpurun_out/r3d/$d "scan_kernel" | grep -E "SQ_INSTS_VALU|SQ_INSTS_SALU|SQ_INSTS_LDS|SQ_LDS_BANK|SQ_LDS_IDX|SQ_WAVE_CYCLES|SQ_INSTS_BRANCH|valu_active"; done
