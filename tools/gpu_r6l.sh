# round-6 PMC traffic + kernel traces on the final tree, NeW-CRFs workloads (NYU, KITTI 352x1216, KITTI 352x704)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
RX='gemm_f32_kernel|gemm_glds_kernel|winattn_fwd_kernel|winattn_bwd_kernel'
bash tools/prof_traffic.sh r6l_nyu "$RX" || exit 1
bash tools/prof_traffic.sh r6l_kitti "$RX" --model newcrfs_kitti || exit 1
bash tools/prof_traffic.sh r6l_k704 "$RX" --model newcrfs_kitti704 || exit 1
