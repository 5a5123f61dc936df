# fp32 Depthformer bench line (the bf16 ratio's denominator on the final tree) and the KITTI
# NeW-CRFs GEMM PMC traffic (bench secondary)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --model depthformer --no-secondary --no-cpu-baseline --steps 10 --warmup 3 \
  > gpurun_out/r4y_df32.json 2> gpurun_out/r4y_df32.err || { tail -20 gpurun_out/r4y_df32.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r4y_df32.json').read().strip().splitlines()[-1]);print('depthformer fp32',d['value'],d['ms_per_step'],d['roofline']['frac'])"
bash tools/prof_round.sh r4_kitti --model newcrfs_kitti --no-secondary || exit 1
echo kitti prof done
