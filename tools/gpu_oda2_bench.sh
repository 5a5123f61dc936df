# ODA2 GPU suite + the default bench line (now with every single-GPU BASELINE config as a secondary)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_oda2_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/oda2_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/oda2_tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_sec.log 2>&1 || { tail -30 gpurun_out/bench_sec.log; exit 1; }
grep '^{"metric' gpurun_out/bench_sec.log | cut -c1-600
