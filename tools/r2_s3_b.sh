set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_head.py 480 640 2 > gpurun_out/diag_head_480.log 2>&1 || { tail -30 gpurun_out/diag_head_480.log; exit 1; }
cat gpurun_out/diag_head_480.log
timeout -k 10 300 python -u tools/diag_head.py 352 384 2 > gpurun_out/diag_head_352.log 2>&1 || { tail -30 gpurun_out/diag_head_352.log; exit 1; }
cat gpurun_out/diag_head_352.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_fullsize_grads_gpu.py::test_adabins_nyu_480x640_train_step_gradients > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_fp32.log 2>&1 || { tail -20 gpurun_out/bench_fp32.log; exit 1; }
grep '^{"metric' gpurun_out/bench_fp32.log
timeout -k 10 400 python -u bench.py --precision fp32e --no-cpu-baseline > gpurun_out/bench_fp32e.log 2>&1 || { tail -20 gpurun_out/bench_fp32e.log; exit 1; }
grep '^{"metric' gpurun_out/bench_fp32e.log
timeout -k 10 300 python -u tools/m16_bench.py > gpurun_out/m16_bench.log 2>&1 || { cat gpurun_out/m16_bench.log; exit 1; }
cat gpurun_out/m16_bench.log
