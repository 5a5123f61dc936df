# after removing the GEMM-epilogue dropout: fusion tests + A/B against the pre-dropout build on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dropout_fused_gpu.py \
  tests/test_conv_skip_gpu.py tests/test_gemm_b16_gpu.py > gpurun_out/r6s_tests.log 2>&1; trc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r6s_tests.log | tail -5
[ $trc -eq 0 ] || exit $trc
A="--no-cpu-baseline --no-secondary --steps 10 --warmup 3"
D="--model depthformer_bf16 --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
OLD="MDEMI_LIB=tools/study/pre_drop/libmdemi.so MDEMI_FUSE_DROPOUT=0"
bash tools/gpu_ab.sh r6s "nyu:-:$A" "nyu_old:$OLD:$A" "df:-:$D" "df_old:$OLD:$D" "nyu2:-:$A" "nyu_old2:$OLD:$A" \
  "df2:-:$D" "df_old2:$OLD:$D"
