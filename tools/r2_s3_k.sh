# fp32 256-row variants: bit-identity vs the other variants, then the whole suite and the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ext_kernels_gpu.py -q -k "variants_bit_identical or two_level" --timeout 120 --timeout-method thread > gpurun_out/var_tests.log 2>&1 || { tail -30 gpurun_out/var_tests.log; exit 1; }
tail -1 gpurun_out/var_tests.log
timeout -k 10 300 python -u tools/m16_bench.py > gpurun_out/m16_bench_v.log 2>&1 || { tail -5 gpurun_out/m16_bench_v.log; exit 1; }
cut -c1-75 gpurun_out/m16_bench_v.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_v.log 2>&1 || { tail -20 gpurun_out/bench_v.log; exit 1; }
grep '^{"metric' gpurun_out/bench_v.log | cut -c1-420
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_v.log 2>&1; rc=$?
grep -E "FAIL|passed|failed" gpurun_out/gpu_tests_v.log | tail -10
exit $rc
