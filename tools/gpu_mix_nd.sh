set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LEGS="mixed reorder_flat_fixed" TESTS=0 bash tools/ab_flat.sh ${1:-r5mixnd} base mix mixnd
