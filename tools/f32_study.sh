# Build kernel-study variants of libmdemi (the fp32 GEMM family with -D flags) into tools/study/<tag>/libmdemi.so:
#   bash tools/f32_study.sh <tag> [-DFLAG ...]      (CPU; then MDEMI_LIB=tools/study/<tag>/libmdemi.so on the GPU box)
set -e
TAG=$1; shift
cd $(dirname $0)/../monocular-depth-estimation_amd/csrc
OUT=../../tools/study/$TAG
mkdir -p $OUT
for s in gemm_f32_inst0 gemm_f32_inst1 gemm_f32_inst2 gemm_f32_inst3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -Wall -Wno-unused-function \
    -munsafe-fp-atomics -ffp-contract=fast "$@" -c $s.hip -o $OUT/$s.o &
done
wait
OBJS=$(ls build/*.o | grep -v gemm_f32_inst)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $OUT/gemm_f32_inst*.o -o $OUT/libmdemi.so
echo built $OUT/libmdemi.so
