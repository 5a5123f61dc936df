# Depthformer v8 bf16 + hipGraph step (configs[4]) and fp32, with a kernel trace of the bf16 step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --model depthformer_bf16 > gpurun_out/bench_dfbf16.log 2>&1 || { tail -30 gpurun_out/bench_dfbf16.log; exit 1; }
tail -1 gpurun_out/bench_dfbf16.log
timeout -k 10 400 python -u bench.py --model depthformer --no-cpu-baseline > gpurun_out/bench_df32.log 2>&1 || { tail -30 gpurun_out/bench_df32.log; exit 1; }
tail -1 gpurun_out/bench_df32.log
timeout -k 10 400 python -u bench.py --model adabins --no-cpu-baseline > gpurun_out/bench_ada.log 2>&1 || { tail -30 gpurun_out/bench_ada.log; exit 1; }
tail -1 gpurun_out/bench_ada.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dfbf16_trace -o run --output-format csv -- python3 bench.py --model depthformer_bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/dfbf16_trace.log 2>&1 || { tail -30 gpurun_out/dfbf16_trace.log; exit 1; }
echo done
