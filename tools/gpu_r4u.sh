# in-kernel BatchNorm combine threshold A/B (MDEMI_BN_INLINE_MAX = max partial blocks x channels)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for th in 0 4096 65536 0; do
for m in depthformer_bf16 adabins; do
MDEMI_BN_INLINE_MAX=$th timeout -k 10 300 python -u bench.py --model $m --no-secondary --no-cpu-baseline --no-roofline --steps 10 --warmup 3 \
  > gpurun_out/r4u_${m}_$th.json 2> gpurun_out/r4u_${m}_$th.err || { tail -20 gpurun_out/r4u_${m}_$th.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r4u_${m}_$th.json').read().strip().splitlines()[-1]);print('$m $th',d['value'],d['ms_per_step'])"
done; done
