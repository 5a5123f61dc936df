# Round-4 profile set of the current tree: NeW-CRFs NYU kernel trace + GEMM PMC traffic (both fp32
# GEMM templates), window-attention trace + PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/prof_round.sh r4_newcrfs --no-secondary || exit 1
bash tools/prof_winattn.sh r4_wa || exit 1
echo prof_r4 done
