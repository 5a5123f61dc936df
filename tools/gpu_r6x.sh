# conv weight re-layout writing its bf16 copy; the conv_pw skip's backward node counted as a GEMM consumer
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_conv_skip_gpu.py \
  tests/test_dropout_fused_gpu.py tests/test_gemm_b16_gpu.py tests/test_bf16_graph_gpu.py tests/test_kernels_gpu.py \
  > gpurun_out/r6x_tests.log 2>&1; trc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r6x_tests.log | tail -5
[ $trc -eq 0 ] || exit $trc
D="--model depthformer_bf16 --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
AD="--model adabins --no-cpu-baseline --no-roofline --steps 5 --warmup 2"
bash tools/gpu_ab.sh r6x "df:-:$D" "df_noskip:MDEMI_CONV_SKIP=0:$D" "df2:-:$D" "df_noskip2:MDEMI_CONV_SKIP=0:$D" \
  "ada:-:$AD" "ada_noskip:MDEMI_CONV_SKIP=0:$AD" || exit 1
timeout -k 10 300 python -u tools/op_sources.py mdemi_cast_bf16 > gpurun_out/r6x_op_sources.txt 2>&1 || exit 1
grep -c cast gpurun_out/r6x_op_sources.txt; grep cast gpurun_out/r6x_op_sources.txt | awk '{s+=$1} END {print "casts per step:", s}'
