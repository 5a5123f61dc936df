# A/B: fp32 inline vs separate split-K combine (NYU, AdaBins), bf16 default vs inline (Depthformer)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
A="--no-cpu-baseline --no-secondary --steps 10 --warmup 3"
D="--model depthformer_bf16 --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
AD="--model adabins --batch 16 --no-cpu-baseline --no-roofline --steps 5 --warmup 2"
bash tools/gpu_ab.sh r6j "nyu:-:$A" "nyu_noinl:MDEMI_GEMM_INLINE_REDUCE=0:$A" "df:-:$D" "df_inl:MDEMI_GEMM_INLINE_REDUCE_B16=1:$D" \
  "ada:-:$AD" "ada_noinl:MDEMI_GEMM_INLINE_REDUCE=0:$AD" "nyu2:-:$A" "df2:-:$D"
