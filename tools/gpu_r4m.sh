# the BN-sensitive parity tests after the BN revert, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread \
  "tests/test_bf16_graph_gpu.py::test_depthformer_v8_480x640_bf16_vs_fp64_oracle" \
  tests/test_models_gpu.py::test_adabins_head tests/test_models_gpu.py::test_depthformer_v8_end_to_end_vs_oracle \
  tests/test_kernels_gpu.py -k "batch_norm or freeze_bn or bf16 or adabins_head or end_to_end" \
  > gpurun_out/r4m_tests.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/r4m_tests.log | tail; exit 1; }
tail -2 gpurun_out/r4m_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/r4m_bench.json 2> gpurun_out/r4m_bench.err || { tail -20 gpurun_out/r4m_bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r4m_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline'], d.get('cpu_baseline'))
for k,v in (d.get('secondaries') or {}).items(): print(k, v.get('value'), v.get('ms_per_step'))
print(d.get('hbm_kernels'))"
