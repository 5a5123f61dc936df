# window-attention correctness + kernel trace (run on the GPU box): bash tools/wa_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "window or swin or newcrf or tiny07" -x -q --timeout 200 --timeout-method thread > gpurun_out/wa_tests.log 2>&1 || { tail -30 gpurun_out/wa_tests.log; exit 1; }
tail -2 gpurun_out/wa_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT/tools
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$1_trace -o run --output-format csv -- python3 winattn_bench.py
