set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
NCCL_DEBUG=WARN timeout -k 10 400 python -u -X faulthandler -m pytest tests/test_bf16_graph_gpu.py tests/test_checkpoint_gpu.py tests/test_ddp_gpu.py tests/test_rccl_graph_gpu.py tests/test_models_gpu.py -k "graph or rccl or ddp or checkpoint" -v --timeout 300 --timeout-method thread > gpurun_out/diag2_rccl.log 2>&1; echo "rccl rc=$?"
grep -E "PASSED|FAILED|ERROR|passed|failed|WARN|Abort" gpurun_out/diag2_rccl.log | tail -12
timeout -k 10 600 python -u -m pytest tests/test_fullsize_grads_gpu.py -k adabins -x -q --timeout 550 --timeout-method thread > gpurun_out/diag2_adabins.log 2>&1; echo "adabins rc=$?"
grep -E "^E |passed|failed" gpurun_out/diag2_adabins.log | head -12
