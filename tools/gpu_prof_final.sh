# Round-end profile set of the shipped tree: NeW-CRFs NYU kernel trace + GEMM PMC traffic, window-attention trace + PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/prof_round.sh r3f_newcrfs --no-secondary || exit 1
bash tools/prof_winattn.sh r3f_wa || exit 1
echo prof_final done
