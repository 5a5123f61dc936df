set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -v -s --timeout 900 --timeout-method thread \
  tests/test_bf16_graph_gpu.py -k 480x640 > gpurun_out/r4h_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error|beyond|grad rel-L2" gpurun_out/r4h_tests.log | cut -c1-600 | tail -40
exit $rc
