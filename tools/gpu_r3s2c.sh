set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or drop_scale or linear or mlp" -x -q --timeout 200 --timeout-method thread > gpurun_out/r3s2c_tests.log 2>&1 || { tail -20 gpurun_out/r3s2c_tests.log; exit 1; }
tail -1 gpurun_out/r3s2c_tests.log
A="--no-cpu-baseline --no-secondary"
bash tools/gpu_ab.sh s2c "sc1:-:$A" "plainrel:MDEMI_LIB=tools/study/plainrel/libmdemi.so:$A" "reducek:MDEMI_GEMM_INLINE_REDUCE=0:$A" "sc1b:-:$A" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fullsize_grads_gpu.py -k adabins -x -q --timeout 550 --timeout-method thread > gpurun_out/r3s2c_adabins.log 2>&1; echo "adabins rc=$?"
grep -E "^E  .*Assert|passed|failed" gpurun_out/r3s2c_adabins.log | head -5
