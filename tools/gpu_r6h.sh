# A/B of split-K / combine / dwconv knobs on the bf16 Depthformer step (one box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
A="--model depthformer_bf16 --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
bash tools/gpu_ab.sh r6h "base:-:$A" "noinl:MDEMI_GEMM_INLINE_REDUCE=0:$A" "t512:MDEMI_SPLIT_TARGET_BLOCKS=512:$A" \
  "t2048:MDEMI_SPLIT_TARGET_BLOCKS=2048:$A" "ty2:MDEMI_DW_TY=2:$A" "mk32:MDEMI_SPLIT_MIN_KTILES=32:$A" "base2:-:$A"
