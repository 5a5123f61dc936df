# round-2 GPU check: new bf16/graph tests, the full GPU suite, two bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bf16_graph_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1; rc=$?
tail -25 gpurun_out/bf16_tests.log
# timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_bf16_graph_gpu.py > gpurun_out/gpu_all.log 2>&1; rc2=$?
rc2=0
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --model depthformer_bf16 --no-cpu-baseline > gpurun_out/bench_dfbf16.log 2>&1 || { tail -30 gpurun_out/bench_dfbf16.log; exit 1; }
tail -1 gpurun_out/bench_dfbf16.log
timeout -k 10 400 python -u bench.py --model depthformer --no-cpu-baseline > gpurun_out/bench_df32.log 2>&1 || { tail -30 gpurun_out/bench_df32.log; exit 1; }
tail -1 gpurun_out/bench_df32.log
exit $rc2
