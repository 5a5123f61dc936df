set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_head.py 480 640 2 testfill > gpurun_out/diag_h_inner.log 2>&1 || { tail -30 gpurun_out/diag_h_inner.log; exit 1; }
sed -n 6,20p gpurun_out/diag_h_inner.log; tail -1 gpurun_out/diag_h_inner.log
MDEMI_GEMM_SPLIT_INNER=1 timeout -k 10 300 python -u tools/diag_head.py 480 640 2 testfill > gpurun_out/diag_h_split.log 2>&1 || { tail -30 gpurun_out/diag_h_split.log; exit 1; }
sed -n 6,20p gpurun_out/diag_h_split.log; tail -1 gpurun_out/diag_h_split.log
