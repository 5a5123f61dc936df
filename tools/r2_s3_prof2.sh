# Final-tree profile set: default bench under rocprofv3 (kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE passes on the GEMM / window-attention / AdamW kernels) -> gpurun_out/r2q_*
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2q_trace -o run --output-format csv -- $B > gpurun_out/r2q_trace.log 2>&1 || { tail -20 gpurun_out/r2q_trace.log; exit 1; }
grep '^{"metric' gpurun_out/r2q_trace.log | cut -c1-300
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'gemm_f32_kernel|winattn|adamw_kernel' -d gpurun_out/r2q_fetch -o run --output-format csv -- $B > gpurun_out/r2q_fetch.log 2>&1 || { tail -20 gpurun_out/r2q_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'gemm_f32_kernel|winattn|adamw_kernel' -d gpurun_out/r2q_write -o run --output-format csv -- $B > gpurun_out/r2q_write.log 2>&1 || { tail -20 gpurun_out/r2q_write.log; exit 1; }
echo profiles done
