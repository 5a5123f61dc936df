set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_relu_kink.py > gpurun_out/diag_kink.log 2>&1 || { tail -8 gpurun_out/diag_kink.log; exit 1; }
tail -3 gpurun_out/diag_kink.log
MDEMI_LIB=tools/study/old/libmdemi.so MDEMI_GEMM_SPLIT_INNER=1 timeout -k 10 300 python -u tools/diag_head.py 480 640 2 testfill > gpurun_out/diag_h_old.log 2>&1 || { tail -30 gpurun_out/diag_h_old.log; exit 1; }
sed -n 9,12p gpurun_out/diag_h_old.log; tail -1 gpurun_out/diag_h_old.log
