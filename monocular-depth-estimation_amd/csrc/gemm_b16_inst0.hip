// Instantiations of the bf16-operand GEMM (gemm_b16_kernel.h), dense layout pairs, and the
// family's kernel selection (gemm_f32.hip mode GEMM_B16).
#include "gemm_b16_kernel.h"

namespace mdemi {

void (*b16_pick_part1(int al, int bl, int v))(GemmParams);

void (*pick_kernel_b16(int al, int bl, int v))(GemmParams) {
  constexpr int KC = MDEMI_L_KCONTIG, MN = MDEMI_L_MNCONTIG;
  if (al == KC && bl == KC) return pick_b16<KC, KC>(v);
  if (al == KC && bl == MN) return pick_b16<KC, MN>(v);
  if (al == MN && bl == KC) return pick_b16<MN, KC>(v);
  if (al == MN && bl == MN) return pick_b16<MN, MN>(v);
  return b16_pick_part1(al, bl, v);
}

}  // namespace mdemi
