# Window-attention kernels under rocprofv3 (run on the GPU box): kernel trace + stats,
# then FETCH_SIZE and WRITE_SIZE in their own --pmc passes restricted to winattn_*.
#   bash tools/prof_winattn.sh <tag>
set -e
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT/tools
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${TAG}_trace -o run --output-format csv -- python3 winattn_bench.py > $O/${TAG}_trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'winattn' -d $O/${TAG}_fetch -o run --output-format csv -- python3 winattn_bench.py > $O/${TAG}_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'winattn' -d $O/${TAG}_write -o run --output-format csv -- python3 winattn_bench.py > $O/${TAG}_write.log 2>&1
echo profiles done
