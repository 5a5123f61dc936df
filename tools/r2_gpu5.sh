# f32e (fp32 image, split at fragment read): accuracy tests, bench lines fp32e + bf16 DFv8, AdaBins full-size test
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_f32e_gpu.py tests/test_bf16_graph_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/f32e_tests.log 2>&1; rc=$?
tail -15 gpurun_out/f32e_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --precision fp32e --no-cpu-baseline --no-secondary > gpurun_out/bench_f32e.log 2>&1 || { tail -30 gpurun_out/bench_f32e.log; exit 1; }
tail -1 gpurun_out/bench_f32e.log
timeout -k 10 400 python -u bench.py --model depthformer_bf16 --no-cpu-baseline > gpurun_out/bench_dfbf16.log 2>&1 || { tail -30 gpurun_out/bench_dfbf16.log; exit 1; }
tail -1 gpurun_out/bench_dfbf16.log
timeout -k 10 600 python -u -m pytest tests/test_fullsize_grads_gpu.py -q --timeout 500 --timeout-method thread -k adabins > gpurun_out/fullsize_ada.log 2>&1; rc2=$?
tail -15 gpurun_out/fullsize_ada.log
exit $((rc + rc2))
