# split-K target-workgroups A/B (MDEMI_SPLIT_TARGET_BLOCKS) on the Depthformer bf16, NeW-CRFs and AdaBins steps
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for tb in 512 768 1024; do
for m in newcrfs adabins; do
MDEMI_SPLIT_TARGET_BLOCKS=$tb timeout -k 10 300 python -u bench.py --model $m --no-secondary --no-cpu-baseline --no-roofline --steps 10 --warmup 3 \
  > gpurun_out/r4s_${m}_$tb.json 2> gpurun_out/r4s_${m}_$tb.err || { tail -20 gpurun_out/r4s_${m}_$tb.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r4s_${m}_$tb.json').read().strip().splitlines()[-1]);print('$m $tb',d['value'],d['ms_per_step'])"
done; done
