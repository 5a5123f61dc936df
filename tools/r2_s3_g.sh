# Full GPU suite + smoke + bench lines (default NeW-CRFs, AdaBins with bin-head GB/s)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_f.log 2>&1; rc=$?
grep -E "FAIL|passed|failed" gpurun_out/gpu_tests_f.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_f.log 2>&1 || { tail -20 gpurun_out/smoke_f.log; exit 1; }
tail -1 gpurun_out/smoke_f.log
timeout -k 10 400 python -u bench.py --model adabins --no-cpu-baseline > gpurun_out/bench_adabins_f.log 2>&1 || { tail -20 gpurun_out/bench_adabins_f.log; exit 1; }
grep '^{"metric' gpurun_out/bench_adabins_f.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_f.log 2>&1 || { tail -20 gpurun_out/bench_f.log; exit 1; }
grep '^{"metric' gpurun_out/bench_f.log
timeout -k 10 400 python -u bench.py --model depthformer --no-cpu-baseline > gpurun_out/bench_dfv8_g.log 2>&1 || { tail -20 gpurun_out/bench_dfv8_g.log; exit 1; }
grep '^{"metric' gpurun_out/bench_dfv8_g.log
timeout -k 10 400 python -u bench.py --model depthformer_bf16 --no-cpu-baseline > gpurun_out/bench_dfv8bf16_g.log 2>&1 || { tail -20 gpurun_out/bench_dfv8bf16_g.log; exit 1; }
grep '^{"metric' gpurun_out/bench_dfv8bf16_g.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-include-regex gemm_f32_kernel -d gpurun_out/f32_pmc1 -o run --output-format csv -- python3 tools/m16_bench.py 3 > gpurun_out/f32_pmc1.log 2>&1 || { tail -5 gpurun_out/f32_pmc1.log; exit 1; }
echo pmc done
