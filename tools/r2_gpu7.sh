set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for t in base ablate; do
  M16_KK_ONLY=1 MDEMI_LIB=tools/study/$t/libmdemi.so timeout -k 10 200 python -u tools/m16_bench.py > gpurun_out/study_$t.log 2>&1 || { cat gpurun_out/study_$t.log; exit 1; }
  echo "== $t"; cat gpurun_out/study_$t.log
done
timeout -k 10 300 python -u -m pytest tests/test_checkpoint_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/ck.log 2>&1; tail -3 gpurun_out/ck.log
