# PMC traffic + traces of AdaBins and configs[4] on the final library
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/prof_traffic.sh r6ab_ada 'gemm_f32_kernel|gemm_glds_kernel|binhead_nhwc' --model adabins || exit 1
bash tools/prof_traffic.sh r6ab_df 'gemm_b16_kernel' --model depthformer_bf16 || exit 1
echo r6ab done
