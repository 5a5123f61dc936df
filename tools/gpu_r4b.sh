# round 4: NeW-CRFs bench (no secondaries) on the glds-GEMM tree, then the slow full-size parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err
rc=$?
tail -3 gpurun_out/r4b_bench.json
[ $rc -eq 0 ] || { tail -20 gpurun_out/r4b_bench.err; exit $rc; }
timeout -k 10 1000 python -u -m pytest -v -s --timeout 600 --timeout-method thread \
  tests/test_fullsize_grads_gpu.py tests/test_bf16_graph_gpu.py::test_depthformer_v8_480x640_bf16_vs_fp64_oracle \
  tests/test_models_gpu.py::test_depthformer_v8_end_to_end_vs_oracle tests/test_oda2_gpu.py::test_oda2_model_end_to_end \
  > gpurun_out/r4b_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert|configs\[4\]" gpurun_out/r4b_tests.log | tail -40
exit $rc
