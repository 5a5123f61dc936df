# final tree: the whole GPU suite, smoke, configs[4] twice, the bf16 cast census
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_rccl_graph_gpu.py tests/test_models_gpu.py tests/test_bf16_graph_gpu.py tests/test_gemm_b16_gpu.py -v --timeout 600 --timeout-method thread > gpurun_out/r6y_tests.log 2>&1; trc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r6y_tests.log | tail -6
[ $trc -eq 0 ] || exit $trc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6y_smoke.log 2>&1 || { tail -20 gpurun_out/r6y_smoke.log; exit 1; }
tail -1 gpurun_out/r6y_smoke.log
D="--model depthformer_bf16 --no-cpu-baseline --no-roofline --steps 10 --warmup 3"
bash tools/gpu_ab.sh r6y "df:-:$D" "df2:-:$D" || exit 1
timeout -k 10 300 python -u tools/op_sources.py mdemi_cast_bf16 > gpurun_out/r6y_op_sources.txt 2>&1 || exit 1
grep cast gpurun_out/r6y_op_sources.txt | awk '{s+=$1} END {print "casts per step:", s}'
