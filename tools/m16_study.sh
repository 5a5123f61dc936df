# Build kernel-study variants of libmdemi (gemm_mfma16 with -D flags) into tools/study/<tag>/libmdemi.so:
#   bash tools/m16_study.sh <tag> [-DFLAG ...]      (CPU; then MDEMI_LIB=tools/study/<tag>/libmdemi.so on the GPU box)
set -e
TAG=$1; shift
cd $(dirname $0)/../monocular-depth-estimation_amd/csrc
OUT=../../tools/study/$TAG
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -Wall -Wno-unused-function \
  -munsafe-fp-atomics -ffp-contract=fast "$@" -c gemm_mfma16.hip -o $OUT/gemm_mfma16.o
OBJS=$(ls build/*.o | grep -v gemm_mfma16)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $OUT/gemm_mfma16.o -o $OUT/libmdemi.so
echo built $OUT/libmdemi.so
