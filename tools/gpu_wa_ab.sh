# window-attention A/B: shipped library vs tools/study/<tag> builds (same box); parity test first
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "window_attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/wa_tests.log 2>&1 || { tail -20 gpurun_out/wa_tests.log; exit 1; }
tail -1 gpurun_out/wa_tests.log
for t in lib "$@" lib; do
  L=monocular-depth-estimation_amd/mdemi/libmdemi.so; [ $t = lib ] || L=tools/study/$t/libmdemi.so
  MDEMI_LIB=$L timeout -k 10 200 python -u tools/winattn_bench.py > gpurun_out/wa_$t.log 2>&1 || { tail -20 gpurun_out/wa_$t.log; exit 1; }
  echo "$t $(tail -1 gpurun_out/wa_$t.log)"
done
