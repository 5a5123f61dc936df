# round 4: targeted GPU tests (new parity tests, glds GEMM variants), then a GEMM study
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py::test_gemm_variants_bit_identical tests/test_kernels_gpu.py::test_gemm_tail_split \
  tests/test_kernels_gpu.py::test_gemm_inline_combine_matches_reduce_kernel \
  tests/test_oda2_gpu.py::test_ordered_window_attention_kernel tests/test_checkpoint_gpu.py \
  tests/test_rccl_graph_gpu.py > gpurun_out/r4a_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r4a_tests.log
[ $rc -eq 0 ] || exit $rc
SHAPES="9600x3072x768:fwd,9600x768x3072:fwd,9600x768x3072:dgrad,9600x2304x768:fwd,38400x1536x384:fwd,153600x768x192:fwd,3072x768x9600:wgrad" \
  timeout -k 10 300 python -u tools/gemm_study.py lib 0,1,3,4,5,6,7,8,9,10,11 > gpurun_out/r4a_gemm_study.log 2>&1
rc=$?
grep TF gpurun_out/r4a_gemm_study.log
exit $rc
