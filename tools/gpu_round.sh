# Full check of the tree on a GPU box: GPU suite, smoke, default bench.
# usage: bash tools/gpu_round.sh <tag> [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-run}; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/gpu_tests_$tag.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
grep '^{"metric' gpurun_out/bench_$tag.log
