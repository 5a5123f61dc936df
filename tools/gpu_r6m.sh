# round-6 PMC traffic + kernel traces on the final tree: AdaBins bs16, Depthformer v8 bf16 (configs[4])
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/prof_traffic.sh r6m_ada 'gemm_f32_kernel|gemm_glds_kernel|binhead_nhwc' --model adabins || exit 1
bash tools/prof_traffic.sh r6m_df 'gemm_b16_kernel' --model depthformer_bf16 || exit 1
timeout -k 10 300 python -u tools/op_sources.py > gpurun_out/r6m_op_sources.txt 2>&1 || { tail -5 gpurun_out/r6m_op_sources.txt; exit 1; }
