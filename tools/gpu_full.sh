# Full check of the tree: whole GPU suite (one process), smoke, default bench line.
#   bash tools/gpu_full.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-run}; shift
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests_$tag.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 500 python -u bench.py "$@" > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
grep '^{"metric' gpurun_out/bench_$tag.log | cut -c1-400
