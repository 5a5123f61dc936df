# eval-mode BN backward tests + configs[4] bf16 parity (train / eval BN), then the round-4
# profile set: NeW-CRFs NYU trace + fp32 GEMM PMC, window attention, Depthformer bf16 trace + m16 PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "batch_norm or freeze_bn" > gpurun_out/r4j_bn.log 2>&1 || { tail -20 gpurun_out/r4j_bn.log; exit 1; }
tail -2 gpurun_out/r4j_bn.log
timeout -k 10 900 python -u -m pytest -v -s --timeout 800 --timeout-method thread \
  tests/test_bf16_graph_gpu.py -k 480x640 > gpurun_out/r4j_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error|beyond|grad rel-L2|noise" gpurun_out/r4j_tests.log | cut -c1-400 | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/prof_round.sh r4_newcrfs --no-secondary || exit 1
bash tools/prof_winattn.sh r4_wa || exit 1
KREGEX='gemm_m16_kernel' bash tools/prof_round.sh r4_dfbf16 --model depthformer_bf16 --no-secondary || exit 1
echo prof_r4 done
exit $rc
