# 256-row GEMM variants without scratch + dwconv blocks: tests, studies, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_b16_gpu.py \
  tests/test_kernels_gpu.py tests/test_ext_kernels_gpu.py > gpurun_out/r6e_tests.log 2>&1; trc=$?
tail -3 gpurun_out/r6e_tests.log
[ $trc -eq 0 ] || exit $trc
for ty in 1 4; do
  MDEMI_DW_TY=$ty timeout -k 10 120 python -u tools/dw_bench.py > gpurun_out/r6e_dw_ty$ty.txt 2>&1 || { tail -5 gpurun_out/r6e_dw_ty$ty.txt; exit 1; }
  tail -1 gpurun_out/r6e_dw_ty$ty.txt
done
timeout -k 10 300 python -u tools/b16_variants.py > gpurun_out/r6e_variants.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/r6e_nyu.json 2> gpurun_out/r6e_nyu.err || { tail -5 gpurun_out/r6e_nyu.err; exit 1; }
timeout -k 10 300 python -u bench.py --model depthformer_bf16 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r6e_df.json 2> gpurun_out/r6e_df.err || { tail -5 gpurun_out/r6e_df.err; exit 1; }
python3 -c "
import json
for f in ('r6e_nyu','r6e_df'):
    d=json.loads(open('gpurun_out/'+f+'.json').read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'], d.get('gemm_all',{}).get('gemm_ms_per_step'))"
