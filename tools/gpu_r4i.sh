set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "batch_norm or freeze_bn" > gpurun_out/r4i_bn.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -v -s --timeout 800 --timeout-method thread \
  tests/test_bf16_graph_gpu.py -k 480x640 > gpurun_out/r4i_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r4i_bn.log
grep -E "passed|failed|FAILED|Error|beyond|grad rel-L2" gpurun_out/r4i_tests.log | cut -c1-600 | tail -40
exit $rc
