# All bench workloads on one box (run via gpurun): one JSON line each under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in newcrfs newcrfs_kitti adabins depthformer; do
  timeout -k 10 400 python -u bench.py --model $m > gpurun_out/bench_$m.log 2>&1 || { echo "BENCH $m FAILED"; tail -20 gpurun_out/bench_$m.log; exit 1; }
  grep '^{"metric' gpurun_out/bench_$m.log
done
