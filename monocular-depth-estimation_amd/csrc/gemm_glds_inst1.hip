// Instantiations of the direct-to-LDS fp32 GEMM variants (gemm_glds_kernel.h), layout
// pairs (MNCONTIG, KCONTIG), (MNCONTIG, MNCONTIG).
#include "gemm_glds_kernel.h"

namespace mdemi {

void (*glds_pick_part1(int al, int bl, int v))(GemmParams) {
  if (al == MDEMI_L_MNCONTIG && bl == MDEMI_L_KCONTIG) return pick_glds<MDEMI_L_MNCONTIG, MDEMI_L_KCONTIG>(v);
  if (al == MDEMI_L_MNCONTIG && bl == MDEMI_L_MNCONTIG) return pick_glds<MDEMI_L_MNCONTIG, MDEMI_L_MNCONTIG>(v);
  return nullptr;
}

}  // namespace mdemi
