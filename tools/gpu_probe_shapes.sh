# Per-shape GEMM timing inside one real train step, for the workloads given (default: the
# bf16 Depthformer step and the NeW-CRFs NYU step):  bash tools/gpu_probe_shapes.sh <tag> [model ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-probe}; shift
models=${@:-depthformer_bf16 newcrfs}
for m in $models; do
  timeout -k 10 300 python -u tools/gemm_shapes.py --model $m > gpurun_out/${tag}_shapes_$m.txt 2>&1 || { tail -20 gpurun_out/${tag}_shapes_$m.txt; exit 1; }
  head -30 gpurun_out/${tag}_shapes_$m.txt
done
