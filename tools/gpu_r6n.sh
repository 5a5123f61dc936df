# dropout fused into GEMM epilogues / the attention softmax, conv_pw skip, DDP bucket rebuild: tests, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dropout_fused_gpu.py \
  tests/test_conv_skip_gpu.py tests/test_rccl_graph_gpu.py tests/test_gemm_b16_gpu.py tests/test_bf16_graph_gpu.py \
  > gpurun_out/r6n_tests.log 2>&1; trc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r6n_tests.log | tail -5
[ $trc -eq 0 ] || exit $trc
A="--no-cpu-baseline --no-secondary --steps 10 --warmup 3"
D="--model depthformer_bf16 --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
AD="--model adabins --no-cpu-baseline --no-roofline --steps 5 --warmup 2"
bash tools/gpu_ab.sh r6n "df:-:$D" "df_nofuse:MDEMI_FUSE_DROPOUT=0 MDEMI_CONV_SKIP=0:$D" "df2:-:$D" \
  "df_noskip:MDEMI_CONV_SKIP=0:$D" "df_nodrop:MDEMI_FUSE_DROPOUT=0:$D" "ada:-:$AD" "ada_noskip:MDEMI_CONV_SKIP=0:$AD" "nyu:-:$A"
