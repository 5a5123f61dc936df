# Profile set for one bench workload (run on the GPU box):
#   bash tools/prof_round.sh <tag> [bench args...]
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in their own --pmc passes
# (GEMM kernels + adamw only: an unrestricted WRITE_SIZE pass segfaults inside
# the profiler on this image), then the per-family traffic table.
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
KRE=${KREGEX:-'gemm_f32_kernel|gemm_glds_kernel|adamw_kernel'}
B="python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o run --output-format csv -- $B > gpurun_out/${TAG}_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d gpurun_out/${TAG}_fetch -o run --output-format csv -- $B > gpurun_out/${TAG}_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d gpurun_out/${TAG}_write -o run --output-format csv -- $B > gpurun_out/${TAG}_write.log 2>&1
echo profiles done
