# Round-2 state check: full GPU suite, smoke, default bench (fp32 and fp32e), 16-bit GEMM microbench
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_fp32.log 2>&1 || { tail -20 gpurun_out/bench_fp32.log; exit 1; }
grep '^{"metric' gpurun_out/bench_fp32.log
timeout -k 10 400 python -u bench.py --precision fp32e --no-cpu-baseline > gpurun_out/bench_fp32e.log 2>&1 || { tail -20 gpurun_out/bench_fp32e.log; exit 1; }
grep '^{"metric' gpurun_out/bench_fp32e.log
timeout -k 10 300 python -u tools/m16_bench.py > gpurun_out/m16_bench.log 2>&1 || { cat gpurun_out/m16_bench.log; exit 1; }
cat gpurun_out/m16_bench.log
