# round 4: bf16 configs[4] gradient diagnostics, then a bench with the family breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
MDEMI_BF16_DIAG=1 timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread \
  tests/test_bf16_graph_gpu.py::test_depthformer_v8_480x640_bf16_vs_fp64_oracle > gpurun_out/r4e_diag.log 2>&1
rc=$?
grep -E "grad rel-L2|PASS|FAIL|Error" gpurun_out/r4e_diag.log | head -50
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/r4e_bench.json 2> gpurun_out/r4e_bench.err
rc=$?
python - <<'PY'
import json
d=json.loads(open("gpurun_out/r4e_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["achieved"])
print(json.dumps(d["gemm_all"]))
PY
exit $rc
