# whole GPU suite, then the Depthformer bf16 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
  > gpurun_out/gpu_full.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_full.log | tail -12
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4n.sh
