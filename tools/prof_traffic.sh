# rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (each in its own run, as the
# MI355X guide prescribes) of one bench workload, restricted to the kernels of interest:
#   bash tools/prof_traffic.sh <tag> '<kernel regex>' [bench args...]
# then locally: python tools/pmc_traffic.py gpurun_out/<tag>_fetch gpurun_out/<tag>_write 2 <workload> profiles/traffic.json
set -e
TAG=$1; RX=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o run --output-format csv -- $B > gpurun_out/${TAG}_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX|adamw_kernel|adamw_dev_kernel" -d gpurun_out/${TAG}_fetch -o run --output-format csv -- $B > gpurun_out/${TAG}_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX|adamw_kernel|adamw_dev_kernel" -d gpurun_out/${TAG}_write -o run --output-format csv -- $B > gpurun_out/${TAG}_write.log 2>&1
echo "profiles $TAG done"
