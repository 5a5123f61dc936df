# Build window-attention study variants of libmdemi (winattn.hip with -D flags) into tools/study/<tag>/:
#   bash tools/wa_study.sh <tag> [-DFLAG ...]     (CPU; then tools/gpu_wa_ab.sh <tag> ... on the GPU box)
set -e
TAG=$1; shift
cd $(dirname $0)/../monocular-depth-estimation_amd/csrc
OUT=../../tools/study/$TAG
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -Wall -Wno-unused-function \
  -munsafe-fp-atomics -ffp-contract=fast "$@" -c winattn.hip -o $OUT/winattn.o
OBJS=$(ls build/*.o | grep -v winattn)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $OUT/winattn.o -o $OUT/libmdemi.so
echo built $OUT/libmdemi.so
