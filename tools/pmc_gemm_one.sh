# PMC passes over one GEMM shape (tools/gemm_one.py): bash tools/pmc_gemm_one.sh <variant> <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_$2
G="python3 tools/gemm_one.py 9600 3072 768 $1 fwd 10"
timeout -k 10 60 $G > gpurun_out/pmc_$2/time.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex gemm_f32_kernel -d gpurun_out/pmc_$2/p1 -o run --output-format csv -- $G > gpurun_out/pmc_$2/p1.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex gemm_f32_kernel -d gpurun_out/pmc_$2/p2 -o run --output-format csv -- $G > gpurun_out/pmc_$2/p2.log 2>&1 || exit 3
