# A/B of the epilogue-dropout build against the round-6 build before it (tools/study/pre_drop, same tree
# otherwise; dropout fusion off in both arms), then PMC traffic + traces of AdaBins and configs[4]
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
A="--no-cpu-baseline --no-secondary --steps 10 --warmup 3"
D="--model depthformer_bf16 --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
OLD="MDEMI_LIB=tools/study/pre_drop/libmdemi.so MDEMI_FUSE_DROPOUT=0"
bash tools/gpu_ab.sh r6q "nyu:-:$A" "nyu_old:$OLD:$A" "nyu2:-:$A" "nyu_old2:$OLD:$A" \
  "df_nofuse:MDEMI_FUSE_DROPOUT=0:$D" "df_old:$OLD:$D" || exit 1
bash tools/prof_traffic.sh r6m_ada 'gemm_f32_kernel|gemm_glds_kernel|binhead_nhwc' --model adabins || exit 1
bash tools/prof_traffic.sh r6m_df 'gemm_b16_kernel' --model depthformer_bf16 || exit 1
timeout -k 10 300 python -u tools/op_sources.py > gpurun_out/r6m_op_sources.txt 2>&1 || { tail -5 gpurun_out/r6m_op_sources.txt; exit 1; }
