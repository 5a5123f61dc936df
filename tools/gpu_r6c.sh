# deep-pipeline bf16 GEMM: bit-identity tests + variant study
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_b16_gpu.py \
  > gpurun_out/r6c_tests.log 2>&1; trc=$?
tail -3 gpurun_out/r6c_tests.log
[ $trc -eq 0 ] || exit $trc
timeout -k 10 300 python -u tools/b16_variants.py > gpurun_out/r6c_variants.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6c_variants.txt
exit $rc
