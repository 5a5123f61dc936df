# round-6 PMC traffic for the two --model lines the default bench does not carry: ODA2 and fp32 Depthformer v8
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/prof_traffic.sh r6aa_oda2 'gemm_f32_kernel|gemm_glds_kernel|winattn_fwd_kernel|winattn_bwd_kernel' --model oda2 || exit 1
bash tools/prof_traffic.sh r6aa_df32 'gemm_f32_kernel|gemm_glds_kernel' --model depthformer || exit 1
echo r6aa done
