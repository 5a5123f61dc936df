# round-6 probe: bf16 Depthformer and NYU kernel traces (per-grid GEMM shapes) + the changed tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_rccl_graph_gpu.py tests/test_bf16_graph_gpu.py -k "quiesce or readiness or 480x640_bf16_vs" \
  > gpurun_out/r6b_tests.log 2>&1; trc=$?
grep -E "passed|failed|output |attention calls|Error|assert" gpurun_out/r6b_tests.log | tail -30
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6b_df -o run --output-format csv -- python3 bench.py --model depthformer_bf16 --steps 5 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r6b_df.log 2>&1 || exit 1
python3 tools/step_breakdown.py gpurun_out/r6b_df 3 70 --by-grid > gpurun_out/r6b_df_breakdown.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6b_nyu -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-secondary > gpurun_out/r6b_nyu.log 2>&1 || exit 1
python3 tools/step_breakdown.py gpurun_out/r6b_nyu 2 70 --by-grid > gpurun_out/r6b_nyu_breakdown.txt 2>&1 || true
head -3 gpurun_out/r6b_df_breakdown.txt gpurun_out/r6b_nyu_breakdown.txt
exit $trc
