# round 3: tail split + inline split-K combine + fused DropPath: kernel tests, RCCL graph tests, GEMM study, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_rccl_graph_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3s2a_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r3s2a_tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
export SHAPES=7680x3072x768:fwd,9600x3072x768:fwd,9600x768x3072:fwd,9600x768x3072:dgrad,9600x2304x768:fwd,38400x1536x384:fwd
timeout -k 10 200 python -u tools/gemm_study.py tail 1,4,6 > gpurun_out/r3s2a_study.log 2>&1 || exit 1
grep TF gpurun_out/r3s2a_study.log
MDEMI_GEMM_TAIL_SPLIT=0 timeout -k 10 200 python -u tools/gemm_study.py notail 4 > gpurun_out/r3s2a_study0.log 2>&1 || exit 1
grep TF gpurun_out/r3s2a_study0.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3s2a_bench.log 2>&1 || { tail -20 gpurun_out/r3s2a_bench.log; exit 1; }
grep '^{"metric' gpurun_out/r3s2a_bench.log | cut -c1-300
