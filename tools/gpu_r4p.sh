# BN kernel tests + Depthformer bf16 / AdaBins bench lines (BN partial-pass unroll A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_ext_kernels_gpu.py \
  -k "batch_norm or freeze_bn or group_norm or chnorm" > gpurun_out/r4p_tests.log 2>&1 || { tail -30 gpurun_out/r4p_tests.log; exit 1; }
tail -1 gpurun_out/r4p_tests.log
for m in depthformer_bf16 adabins; do
timeout -k 10 300 python -u bench.py --model $m --no-secondary --no-cpu-baseline --no-roofline --steps 10 --warmup 3 \
  > gpurun_out/r4p_$m.json 2> gpurun_out/r4p_$m.err || { tail -20 gpurun_out/r4p_$m.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r4p_$m.json').read().strip().splitlines()[-1]);print('$m',d['value'],d['ms_per_step'])"
done
