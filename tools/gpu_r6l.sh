# round-6 PMC traffic + kernel traces on the final tree, NeW-CRFs workloads (NYU, KITTI 352x1216, KITTI 352x704),
# then a kernel trace of configs[4] to cross-check the line's event timing of its small GEMMs
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
RX='gemm_f32_kernel|gemm_glds_kernel|winattn_fwd_kernel|winattn_bwd_kernel'
bash tools/prof_traffic.sh r6l_nyu "$RX" || exit 1
bash tools/prof_traffic.sh r6l_kitti "$RX" --model newcrfs_kitti || exit 1
bash tools/prof_traffic.sh r6l_k704 "$RX" --model newcrfs_kitti704 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6l_df_trace -o run --output-format csv -- \
  python3 bench.py --model depthformer_bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary \
  > gpurun_out/r6l_df_trace.log 2>&1 || exit 1
echo r6l done
