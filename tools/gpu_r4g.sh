set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread \
  tests/test_bf16_graph_gpu.py::test_depthformer_v8_480x640_bf16_vs_fp64_oracle > gpurun_out/r4g_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error|configs\[4\]|beyond" gpurun_out/r4g_tests.log | tail -8 | cut -c1-1500
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err || { tail -5 gpurun_out/r4f_bench.err; exit 1; }
timeout -k 10 400 python -u bench.py --model depthformer_bf16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4f_dfbf16.json 2> gpurun_out/r4f_dfbf16.err || { tail -5 gpurun_out/r4f_dfbf16.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r4f_bench.json", "gpurun_out/r4f_dfbf16.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["frac"])
    print({k: (v["tflops"], v["ms_per_step"]) for k, v in d["gemm_all"]["families"].items()})
PY
exit $rc
