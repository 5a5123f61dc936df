set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_fuse.py bf16 > gpurun_out/r6o_diag.txt 2>&1; cat gpurun_out/r6o_diag.txt | tail -30
