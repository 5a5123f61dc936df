# fp32 GEMM study on the GPU box: the shipped library and each tools/study/<tag> build
#   bash tools/gpu_gemm_study.sh <tag...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 python -u tools/gemm_study.py lib > gpurun_out/gemm_study_lib.log 2>&1 || { tail -20 gpurun_out/gemm_study_lib.log; exit 1; }
cat gpurun_out/gemm_study_lib.log | grep TF
for t in "$@"; do
  MDEMI_LIB=tools/study/$t/libmdemi.so timeout -k 10 120 python -u tools/gemm_study.py $t > gpurun_out/gemm_study_$t.log 2>&1 || { tail -20 gpurun_out/gemm_study_$t.log; exit 1; }
  grep TF gpurun_out/gemm_study_$t.log
done
