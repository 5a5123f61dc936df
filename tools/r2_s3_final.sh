# Round-2 final check of the tree: GPU suite, smoke, default bench; kink diagnostic (informational)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1; rc=$?
grep -E "FAIL|passed|failed" gpurun_out/gpu_tests_final.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
grep '^{"metric' gpurun_out/bench_final.log
timeout -k 10 300 python -u tools/diag_relu_kink.py > gpurun_out/diag_kink.log 2>&1; tail -4 gpurun_out/diag_kink.log
