set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_shapes.py --model newcrfs > gpurun_out/r4v_shapes.txt 2>&1 || { tail -20 gpurun_out/r4v_shapes.txt; exit 1; }
head -50 gpurun_out/r4v_shapes.txt
