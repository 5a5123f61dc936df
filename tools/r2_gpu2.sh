# round-2 re-entry GPU check: bf16/graph tests, then the full GPU suite, then the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bf16_graph_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1; rc=$?
tail -25 gpurun_out/bf16_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_bf16_graph_gpu.py > gpurun_out/gpu_all.log 2>&1; rc2=$?
tail -15 gpurun_out/gpu_all.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
exit $((rc + rc2))
