set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_relu_kink.py > gpurun_out/diag_kink.log 2>&1 || { tail -8 gpurun_out/diag_kink.log; exit 1; }
tail -4 gpurun_out/diag_kink.log
