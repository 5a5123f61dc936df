# Round-2 measurement set (run via gpurun): AdaBins and Depthformer-bf16 bench lines, then the
# default NeW-CRFs bench under rocprofv3 (kernel trace + stats, FETCH_SIZE and WRITE_SIZE
# passes on the GEMM, window-attention and AdamW kernels) -> gpurun_out/r2p_*
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for m in adabins depthformer_bf16; do
  timeout -k 10 400 python -u bench.py --model $m > gpurun_out/r2p_bench_$m.log 2>&1 || { echo "BENCH $m FAILED"; tail -20 gpurun_out/r2p_bench_$m.log; exit 1; }
  grep '^{"metric' gpurun_out/r2p_bench_$m.log
done
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p_trace -o run --output-format csv -- $B > gpurun_out/r2p_trace.log 2>&1 || { tail -20 gpurun_out/r2p_trace.log; exit 1; }
grep '^{"metric' gpurun_out/r2p_trace.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'gemm_f32_kernel|winattn|adamw_kernel' -d gpurun_out/r2p_fetch -o run --output-format csv -- $B > gpurun_out/r2p_fetch.log 2>&1 || { tail -20 gpurun_out/r2p_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'gemm_f32_kernel|winattn|adamw_kernel' -d gpurun_out/r2p_write -o run --output-format csv -- $B > gpurun_out/r2p_write.log 2>&1 || { tail -20 gpurun_out/r2p_write.log; exit 1; }
B2="python3 bench.py --model adabins --steps 3 --warmup 2 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'binhead|adamw_kernel' -d gpurun_out/r2p_afetch -o run --output-format csv -- $B2 > gpurun_out/r2p_afetch.log 2>&1 || { tail -20 gpurun_out/r2p_afetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'binhead|adamw_kernel' -d gpurun_out/r2p_awrite -o run --output-format csv -- $B2 > gpurun_out/r2p_awrite.log 2>&1 || { tail -20 gpurun_out/r2p_awrite.log; exit 1; }
echo profiles done
