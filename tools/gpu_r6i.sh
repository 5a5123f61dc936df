# 192-column fp32 tile, bf16 split-K by the reduce kernel + auto split on bf16 1x1 convs: tests + benches + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_gemm_b16_gpu.py tests/test_ext_kernels_gpu.py tests/test_models_gpu.py > gpurun_out/r6i_tests.log 2>&1; trc=$?
tail -3 gpurun_out/r6i_tests.log
[ $trc -eq 0 ] || exit $trc
SHAPES="153600x192x768:fwd,153600x192x768:dgrad,153600x576x192:fwd,768x192x153600:wgrad,153600x192x576:dgrad,9600x3072x768:fwd" \
  timeout -k 10 300 python -u tools/gemm_study.py r6i 4,8,11,12 > gpurun_out/r6i_gemm_study.txt 2>&1 || { tail -5 gpurun_out/r6i_gemm_study.txt; exit 1; }
grep -v amdgpu gpurun_out/r6i_gemm_study.txt
A="--no-cpu-baseline --no-secondary --steps 10 --warmup 3"
D="--model depthformer_bf16 --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
AD="--model adabins --batch 16 --no-cpu-baseline --no-roofline --steps 5 --warmup 2"
bash tools/gpu_ab.sh r6i "nyu:-:$A" "nyu_noinl:MDEMI_GEMM_INLINE_REDUCE=0:$A" "df:-:$D" "df_inl:MDEMI_GEMM_INLINE_REDUCE_B16=1:$D" \
  "ada:-:$AD" "ada_noinl:MDEMI_GEMM_INLINE_REDUCE=0:$AD"
