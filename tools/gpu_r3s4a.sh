# window-attention variants A/B + fp32 GEMM study (no-load / no-sync ceilings) on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_wa_ab.sh wa_old wa_noatom wa_nocols wa_nostore || exit 1
for t in lib noload nosync; do
  L=monocular-depth-estimation_amd/mdemi/libmdemi.so; [ $t = lib ] || L=tools/study/$t/libmdemi.so
  MDEMI_LIB=$L timeout -k 10 200 python -u tools/gemm_study.py $t 0,3,4,8 > gpurun_out/gs_$t.log 2>&1 || { tail -20 gpurun_out/gs_$t.log; exit 1; }
  cat gpurun_out/gs_$t.log
done
