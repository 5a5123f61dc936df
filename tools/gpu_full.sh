# Whole GPU suite + smoke() on the current tree (run on the GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
  > gpurun_out/gpu_full.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_full.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
