# One call: zstd par-kernel PMC mix, then tests / A/B / suite section (gpu_r3_zpar.sh).
# usage: bash scripts/gpu_r3_combo.sh <tag> [section]
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_zpmc.sh $1_zpmc || exit 1
bash scripts/gpu_r3_zpar.sh "$@"
