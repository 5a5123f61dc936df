# parity of the reordered window-attention backward -> A/B vs the 3-workgroup/CU build and the round-start kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_oda2_gpu.py -k "window_attention or gemm or swin or newcrf or oda2" -x -q --timeout 200 --timeout-method thread > gpurun_out/s5_tests.log 2>&1 || { tail -30 gpurun_out/s5_tests.log; exit 1; }
tail -1 gpurun_out/s5_tests.log
MDEMI_LIB=tools/study/wa_occ3/libmdemi.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "window_attention" -x -q --timeout 200 --timeout-method thread > gpurun_out/s5_tests_occ3.log 2>&1 || { tail -30 gpurun_out/s5_tests_occ3.log; exit 1; }
tail -1 gpurun_out/s5_tests_occ3.log
for t in lib wa_occ3 wa_old; do
  L=monocular-depth-estimation_amd/mdemi/libmdemi.so; [ $t = lib ] || L=tools/study/$t/libmdemi.so
  MDEMI_LIB=$L timeout -k 10 200 python -u tools/winattn_bench.py > gpurun_out/wa_$t.log 2>&1 || { tail -20 gpurun_out/wa_$t.log; exit 1; }
  echo "$t $(tail -1 gpurun_out/wa_$t.log)"
done
