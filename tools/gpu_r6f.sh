# SE pooling in the BN sweep, dpooled scale folded, dw lanes: tests + bf16 Depthformer bench + trace breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ext_kernels_gpu.py \
  tests/test_models_gpu.py tests/test_bf16_graph_gpu.py > gpurun_out/r6f_tests.log 2>&1; trc=$?
tail -3 gpurun_out/r6f_tests.log
[ $trc -eq 0 ] || exit $trc
MDEMI_DW_TY=4 timeout -k 10 120 python -u tools/dw_bench.py > gpurun_out/r6f_dw.txt 2>&1 || { tail -5 gpurun_out/r6f_dw.txt; exit 1; }
tail -1 gpurun_out/r6f_dw.txt
timeout -k 10 300 python -u bench.py --model depthformer_bf16 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r6f_df.json 2> gpurun_out/r6f_df.err || { tail -5 gpurun_out/r6f_df.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r6f_df.json').read().strip().splitlines()[-1])
print('df', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('gemm_all',{}).get('gemm_ms_per_step'))"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6f_dft -o run --output-format csv -- python3 bench.py --model depthformer_bf16 --steps 5 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r6f_dft.log 2>&1 || exit 1
python3 tools/step_breakdown.py gpurun_out/r6f_dft 3 70 > gpurun_out/r6f_df_breakdown.txt 2>&1
head -2 gpurun_out/r6f_df_breakdown.txt | cut -c1-300
