set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
AMD_LOG_LEVEL=1 timeout -k 10 400 python -u -m pytest tests/test_bf16_graph_gpu.py tests/test_checkpoint_gpu.py tests/test_ddp_gpu.py tests/test_rccl_graph_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/diag_rccl.log 2>&1; echo "rccl rc=$?"
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/diag_rccl.log | tail -6
timeout -k 10 500 python -u -m pytest tests/test_fullsize_grads_gpu.py -k adabins -x -q --timeout 450 --timeout-method thread > gpurun_out/diag_adabins.log 2>&1; echo "adabins rc=$?"
grep -E "^E |assert|passed|failed" gpurun_out/diag_adabins.log | head -20
bash tools/gpu_wa_ab.sh waold
