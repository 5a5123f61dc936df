set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 800 --timeout-method thread \
  tests/test_bf16_graph_gpu.py -k 480x640 > gpurun_out/r4t_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|noise" gpurun_out/r4t_tests.log | cut -c1-300 | tail -24
exit $rc
