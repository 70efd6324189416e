# round 5 A/B: the flat tier's key table (YSB_BL2_KEYTAB, lib/libysb_hip_kt.so) against base
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LEGS="mixed reorder_flat_fixed mixed_blocks config3_reorder" bash tools/ab_flat.sh r5z base kt
