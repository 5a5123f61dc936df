set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r4p.sh || exit 1
bash tools/gpu_r4w.sh
