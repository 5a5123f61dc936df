# f32e GEMM family: unit accuracy tests, bf16 tests on the new 16-bit kernels, the GPU suite, then benches
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_f32e_gpu.py tests/test_bf16_graph_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/f32e_tests.log 2>&1; rc=$?
tail -40 gpurun_out/f32e_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --precision fp32e --no-cpu-baseline > gpurun_out/bench_f32e.log 2>&1 || { tail -30 gpurun_out/bench_f32e.log; exit 1; }
tail -1 gpurun_out/bench_f32e.log
timeout -k 10 400 python -u bench.py --model depthformer_bf16 --no-cpu-baseline > gpurun_out/bench_dfbf16.log 2>&1 || { tail -30 gpurun_out/bench_dfbf16.log; exit 1; }
tail -1 gpurun_out/bench_dfbf16.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread --deselect tests/test_bf16_graph_gpu.py --deselect tests/test_gemm_f32e_gpu.py > gpurun_out/gpu_all.log 2>&1; rc2=$?
tail -30 gpurun_out/gpu_all.log
exit $((rc + rc2))
