# the last tree of round 6: whole GPU suite, smoke(), the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_final.sh r6z
