// Instantiations of the fp32 GEMM family (gemm_f32_kernel.h), layout pairs
// (MNCONTIG, CONV), (KCONTIG, CONV): one translation unit per pair group so the
// family's many template instances compile in parallel.
#include "gemm_f32_kernel.h"

namespace mdemi {

KernelFn f32_pick_part3(int al, int bl, int aop, int bop, int v) {
  if (al == MDEMI_L_MNCONTIG && bl == MDEMI_L_CONV) return pick_ops<MDEMI_L_MNCONTIG, MDEMI_L_CONV>(aop, bop, v);
  if (al == MDEMI_L_KCONTIG && bl == MDEMI_L_CONV) return pick_ops<MDEMI_L_KCONTIG, MDEMI_L_CONV>(aop, bop, v);
  return nullptr;
}

}  // namespace mdemi
