set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/m16_bench.py > gpurun_out/m16_bench.log 2>&1 || { cat gpurun_out/m16_bench.log; exit 1; }
cat gpurun_out/m16_bench.log
timeout -k 10 600 python -u -m pytest tests/test_gemm_f32e_gpu.py tests/test_bf16_graph_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/f32e_tests.log 2>&1; rc=$?
tail -5 gpurun_out/f32e_tests.log
exit $rc
