set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_augment_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/aug_tests.log 2>&1 ; grep -E "PASS|FAIL|Error" gpurun_out/aug_tests.log | head -30
tail -3 gpurun_out/aug_tests.log
timeout -k 10 300 python -u tools/diag_head.py 480 640 2 enc > gpurun_out/diag_head_enc.log 2>&1 || { tail -30 gpurun_out/diag_head_enc.log; exit 1; }
head -45 gpurun_out/diag_head_enc.log
MDEMI_MATMUL_PRECISION=fp32e timeout -k 10 600 python -u -m pytest tests/test_fullsize_grads_gpu.py tests/test_models_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/fp32e_tests.log 2>&1; echo "fp32e tests rc=$?"
grep -E "PASS|FAIL|passed|failed" gpurun_out/fp32e_tests.log | tail -40
