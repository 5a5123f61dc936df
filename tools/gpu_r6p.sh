# conv_pw skip fusion: tests, then A/B (configs[4], AdaBins) on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_skip_gpu.py \
  tests/test_dropout_fused_gpu.py > gpurun_out/r6p_tests.log 2>&1; trc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r6p_tests.log | tail -5
[ $trc -eq 0 ] || exit $trc
D="--model depthformer_bf16 --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
AD="--model adabins --no-cpu-baseline --no-roofline --steps 5 --warmup 2"
bash tools/gpu_ab.sh r6p "df:-:$D" "df_noskip:MDEMI_CONV_SKIP=0:$D" "ada:-:$AD" "ada_noskip:MDEMI_CONV_SKIP=0:$AD" \
  "df2:-:$D" "df_noskip2:MDEMI_CONV_SKIP=0:$D"
