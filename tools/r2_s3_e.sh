# fp32e (eight plane products) check: 16-bit GEMM microbench, the whole GPU suite under
# MDEMI_MATMUL_PRECISION=fp32e, the full-size tests (both precisions), benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/m16_bench.py > gpurun_out/m16_bench8.log 2>&1 || { cat gpurun_out/m16_bench8.log; exit 1; }
cat gpurun_out/m16_bench8.log
MDEMI_MATMUL_PRECISION=fp32e timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_f32e.log 2>&1; echo "fp32e suite rc=$?"
grep -E "FAIL|passed|failed" gpurun_out/gpu_tests_f32e.log | tail -15
timeout -k 10 400 python -u bench.py --precision fp32e --no-cpu-baseline > gpurun_out/bench_fp32e8.log 2>&1 || { tail -20 gpurun_out/bench_fp32e8.log; exit 1; }
grep '^{"metric' gpurun_out/bench_fp32e8.log
