# A/B on one box: 16-B epilogue on/off, tail split on/off (NeW-CRFs NYU bench, no secondaries)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for cfg in "1 1" "0 1" "1 0" "1 1"; do
  set -- $cfg
  MDEMI_GEMM_EP_VEC=$1 MDEMI_GEMM_TAIL_SPLIT=$2 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab_ep$1_tail$2.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/ab_ep$1_tail$2.json').read().strip().splitlines()[-1])
print('ep_vec=$1 tail=$2', d['value'], d['ms_per_step'], d['gemm_all']['gemm_ms_per_step'], {k:v['tflops'] for k,v in d['gemm_all']['families'].items()})"
done
