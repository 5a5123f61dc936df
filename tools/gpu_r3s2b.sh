set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export SHAPES=8192x3072x768:fwd,9600x3072x768:fwd,9600x768x3072:dgrad,3072x768x9600:wgrad
timeout -k 10 200 python -u tools/gemm_study.py fpf 1,3,4,5,6 > gpurun_out/r3s2b_fpf.log 2>&1 || exit 1
MDEMI_LIB=tools/study/nofpf/libmdemi.so timeout -k 10 200 python -u tools/gemm_study.py nofpf 1,3,4,5,6 > gpurun_out/r3s2b_nofpf.log 2>&1 || exit 1
paste <(grep TF gpurun_out/r3s2b_fpf.log) <(grep TF gpurun_out/r3s2b_nofpf.log | awk '{print $(NF-3), $(NF-1)}')
A="--no-cpu-baseline --no-secondary"
bash tools/gpu_ab.sh s2b "new:-:$A" "nofpf:MDEMI_LIB=tools/study/nofpf/libmdemi.so:$A" "notail:MDEMI_GEMM_TAIL_SPLIT=0:$A" "noinline:MDEMI_GEMM_INLINE_REDUCE=0:$A" "new2:-:$A"
