set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/op_sources.py mdemi_cast_bf16 > gpurun_out/r6w_op_sources.txt 2>&1 || { tail -5 gpurun_out/r6w_op_sources.txt; exit 1; }
grep cast gpurun_out/r6w_op_sources.txt | head -40
