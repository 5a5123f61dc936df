# kernel trace of the Depthformer bf16 captured step (after the gradient-capture change)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4n_dfbf16_trace -o run --output-format csv -- \
  python3 -u bench.py --model depthformer_bf16 --no-secondary --no-cpu-baseline --no-roofline --steps 5 --warmup 2 \
  > gpurun_out/r4n_dfbf16_trace.log 2>&1 || { tail -20 gpurun_out/r4n_dfbf16_trace.log; exit 1; }
python3 tools/step_breakdown.py gpurun_out/r4n_dfbf16_trace 3 60 > gpurun_out/r4n_breakdown.txt
head -40 gpurun_out/r4n_breakdown.txt | cut -c1-160
