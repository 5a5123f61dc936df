# captured-step tests after the grads-None capture change, the Depthformer bf16 bench line,
# and the per-shape GEMM table of the bf16 step
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_bf16_graph_gpu.py tests/test_rccl_graph_gpu.py tests/test_checkpoint_gpu.py -k "not 480x640_bf16_vs" \
  > gpurun_out/r4k_tests.log 2>&1 || { tail -30 gpurun_out/r4k_tests.log; exit 1; }
tail -3 gpurun_out/r4k_tests.log
timeout -k 10 300 python -u bench.py --model depthformer_bf16 --no-secondary --no-cpu-baseline --steps 10 --warmup 3 \
  > gpurun_out/r4k_dfbf16.json 2> gpurun_out/r4k_dfbf16.err || { tail -20 gpurun_out/r4k_dfbf16.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r4k_dfbf16.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"
timeout -k 10 300 python -u tools/gemm_shapes.py --model depthformer_bf16 > gpurun_out/r4k_shapes.txt 2>&1 || { tail -20 gpurun_out/r4k_shapes.txt; exit 1; }
head -40 gpurun_out/r4k_shapes.txt
