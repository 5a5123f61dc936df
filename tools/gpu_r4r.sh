# split-K minimum-rows A/B (MDEMI_SPLIT_MIN_KTILES) on the Depthformer bf16 and NeW-CRFs steps
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for kt in 32 16 8; do
for m in depthformer_bf16 newcrfs; do
MDEMI_SPLIT_MIN_KTILES=$kt timeout -k 10 300 python -u bench.py --model $m --no-secondary --no-cpu-baseline --no-roofline --steps 10 --warmup 3 \
  > gpurun_out/r4r_${m}_$kt.json 2> gpurun_out/r4r_${m}_$kt.err || { tail -20 gpurun_out/r4r_${m}_$kt.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r4r_${m}_$kt.json').read().strip().splitlines()[-1]);print('$m $kt',d['value'],d['ms_per_step'])"
done; done
