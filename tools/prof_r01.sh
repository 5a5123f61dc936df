# Round-1 profile set for the default bench workload (run on the GPU box):
#   kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in their own --pmc passes.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r01_trace -o run --output-format csv -- $B > gpurun_out/r01_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r01_fetch -o run --output-format csv -- $B > gpurun_out/r01_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r01_write -o run --output-format csv -- $B > gpurun_out/r01_write.log 2>&1
