# register-staged bf16 GEMM variants + dwconv block kernels: tests, variant study, dwconv bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_b16_gpu.py \
  tests/test_ext_kernels_gpu.py -k "b16 or bit_identical or dwconv" > gpurun_out/r6d_tests.log 2>&1; trc=$?
tail -3 gpurun_out/r6d_tests.log
[ $trc -eq 0 ] || exit $trc
timeout -k 10 300 python -u tools/b16_variants.py > gpurun_out/r6d_variants.txt 2>&1 || exit 1
for ty in 1 2 4; do
  MDEMI_DW_TY=$ty timeout -k 10 120 python -u tools/dw_bench.py > gpurun_out/r6d_dw_ty$ty.txt 2>&1 || { tail -5 gpurun_out/r6d_dw_ty$ty.txt; exit 1; }
  tail -1 gpurun_out/r6d_dw_ty$ty.txt
done
