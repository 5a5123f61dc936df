// Instantiations of the fp32 GEMM family (gemm_f32_kernel.h), layout pairs
// (CONV, KCONTIG), (CONV, MNCONTIG): one translation unit per pair group so the
// family's many template instances compile in parallel.
#include "gemm_f32_kernel.h"

namespace mdemi {

KernelFn f32_pick_part2(int al, int bl, int aop, int bop, int v) {
  if (al == MDEMI_L_CONV && bl == MDEMI_L_KCONTIG) return pick_ops<MDEMI_L_CONV, MDEMI_L_KCONTIG>(aop, bop, v);
  if (al == MDEMI_L_CONV && bl == MDEMI_L_MNCONTIG) return pick_ops<MDEMI_L_CONV, MDEMI_L_MNCONTIG>(aop, bop, v);
  return nullptr;
}

}  // namespace mdemi
