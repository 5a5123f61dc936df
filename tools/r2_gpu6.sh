# 16-bit GEMM microbench + SQ counters of the f32e kernel on one shape
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/m16_bench.py > gpurun_out/m16_bench.log 2>&1 || { cat gpurun_out/m16_bench.log; exit 1; }
cat gpurun_out/m16_bench.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-include-regex gemm_m16_kernel -d gpurun_out/m16_pmc1 -o run --output-format csv -- python3 tools/m16_bench.py 3 > gpurun_out/m16_pmc1.log 2>&1 || { tail -20 gpurun_out/m16_pmc1.log; exit 1; }
echo pmc done
