// Instantiations of the bf16-operand GEMM (gemm_b16_kernel.h), implicit-im2col layout
// pairs: conv forward (CONV, KCONTIG), data gradient (CONV, MNCONTIG), weight gradient
// (MNCONTIG, CONV).
#include "gemm_b16_kernel.h"

namespace mdemi {

void (*b16_pick_part1(int al, int bl, int v))(GemmParams) {
  constexpr int KC = MDEMI_L_KCONTIG, MN = MDEMI_L_MNCONTIG, CV = MDEMI_L_CONV;
  if (al == CV && bl == KC) return pick_b16<CV, KC>(v);
  if (al == CV && bl == MN) return pick_b16<CV, MN>(v);
  if (al == MN && bl == CV) return pick_b16<MN, CV>(v);
  if (al == KC && bl == CV) return pick_b16<KC, CV>(v);
  return nullptr;
}

}  // namespace mdemi
