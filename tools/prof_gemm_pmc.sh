# SQ / GRBM counters for the fwd GEMM on two model shapes (tools/gemm_sweep.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT/tools
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d ../gpurun_out/gemm_pmc -o run --output-format csv -- python3 gemm_sweep.py 153600x768x192 9600x3072x768 > ../gpurun_out/gemm_pmc.log 2>&1
