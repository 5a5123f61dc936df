# round 4: GEMM epilogue / in-kernel row-sum / DDP-scale-fold checks, bf16 GEMM audit, quick bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_ddp_gpu.py tests/test_bf16_graph_gpu.py -k "not 480x640" > gpurun_out/r4d_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4d_tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bf16_audit.py > gpurun_out/r4d_audit_small.txt 2>&1 || { tail -20 gpurun_out/r4d_audit_small.txt; exit 1; }
cat gpurun_out/r4d_audit_small.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/bf16_audit.py --full > gpurun_out/r4d_audit_full.txt 2>&1 || { tail -20 gpurun_out/r4d_audit_full.txt; exit 1; }
cat gpurun_out/r4d_audit_full.txt | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/r4d_bench.json 2> gpurun_out/r4d_bench.err
rc=$?
tail -1 gpurun_out/r4d_bench.json | cut -c1-900
exit $rc
