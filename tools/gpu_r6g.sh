# fp32 GEMM variant study on the NYU shapes (256-row variants now without scratch) + op sources of the bf16 step
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
SHAPES="9600x3072x768:fwd,9600x3072x768:dgrad,9600x768x3072:fwd,9600x768x3072:dgrad,3072x768x9600:wgrad,768x3072x9600:wgrad,153600x768x192:fwd,153600x192x768:fwd,153600x192x768:dgrad,153600x576x192:fwd,768x192x153600:wgrad" \
  timeout -k 10 300 python -u tools/gemm_study.py r6g 0,1,3,4,5,6,7,8,9,10,11 > gpurun_out/r6g_gemm_study.txt 2>&1 || { tail -5 gpurun_out/r6g_gemm_study.txt; exit 1; }
grep -v amdgpu gpurun_out/r6g_gemm_study.txt | sort -t: -k1,1 -s | head -130
timeout -k 10 300 python -u tools/op_sources.py > gpurun_out/r6g_op_sources.txt 2>&1 || { tail -5 gpurun_out/r6g_op_sources.txt; exit 1; }
grep -v amdgpu gpurun_out/r6g_op_sources.txt | head -80
