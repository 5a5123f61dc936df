# round 4: per-shape GEMM timing (tail split on / off), then the configs[4] bf16 parity test
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_shapes.py > gpurun_out/r4c_shapes_tail1.txt 2>&1 || { tail -20 gpurun_out/r4c_shapes_tail1.txt; exit 1; }
MDEMI_GEMM_TAIL_SPLIT=0 timeout -k 10 300 python -u tools/gemm_shapes.py > gpurun_out/r4c_shapes_tail0.txt 2>&1 || { tail -20 gpurun_out/r4c_shapes_tail0.txt; exit 1; }
head -40 gpurun_out/r4c_shapes_tail1.txt
head -4 gpurun_out/r4c_shapes_tail0.txt
timeout -k 10 900 python -u -m pytest -v -s --timeout 800 --timeout-method thread \
  tests/test_bf16_graph_gpu.py::test_depthformer_v8_480x640_bf16_vs_fp64_oracle > gpurun_out/r4c_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert|configs\[4\]" gpurun_out/r4c_tests.log | tail -20
exit $rc
