# tile-count (wave quantization) study: the same K / N at M giving exact and partial rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export SHAPES=6144x3072x768:fwd,7680x3072x768:fwd,8192x3072x768:fwd,9600x3072x768:fwd,12288x3072x768:fwd,16384x3072x768:fwd,32768x3072x768:fwd
for t in lib noload nosync; do
  L=monocular-depth-estimation_amd/mdemi/libmdemi.so; [ $t = lib ] || L=tools/study/$t/libmdemi.so
  MDEMI_LIB=$L timeout -k 10 120 python -u tools/gemm_study.py $t 1,4,6 > gpurun_out/tail_$t.log 2>&1 || { tail -20 gpurun_out/tail_$t.log; exit 1; }
  grep TF gpurun_out/tail_$t.log
done
