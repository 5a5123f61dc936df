# parity (window attention, GEMM/conv) -> window-attention A/B -> NeW-CRFs bench -> AdaBins GEMM PMC traffic
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "window_attention or gemm or conv or swin or newcrf or linear" -x -q --timeout 200 --timeout-method thread > gpurun_out/s4b_tests.log 2>&1 || { tail -30 gpurun_out/s4b_tests.log; exit 1; }
tail -1 gpurun_out/s4b_tests.log
for t in lib wa_old; do
  L=monocular-depth-estimation_amd/mdemi/libmdemi.so; [ $t = lib ] || L=tools/study/$t/libmdemi.so
  MDEMI_LIB=$L timeout -k 10 200 python -u tools/winattn_bench.py > gpurun_out/wa_$t.log 2>&1 || { tail -20 gpurun_out/wa_$t.log; exit 1; }
  echo "$t $(tail -1 gpurun_out/wa_$t.log)"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > gpurun_out/s4b_bench.log 2>&1 || { tail -20 gpurun_out/s4b_bench.log; exit 1; }
grep '^{"metric' gpurun_out/s4b_bench.log | cut -c1-300
bash tools/prof_traffic.sh s4b_ada 'gemm_f32_kernel' --model adabins || exit 1
MDEMI_LIB=monocular-depth-estimation_amd/mdemi/libmdemi.so timeout -k 10 200 python -u tools/gemm_study.py lib 3,4,8 > gpurun_out/gs_lib.log 2>&1 || { tail -20 gpurun_out/gs_lib.log; exit 1; }
cat gpurun_out/gs_lib.log
