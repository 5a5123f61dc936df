// Instantiations of the 16-bit GEMM family (gemm_mfma16_kernel.h), layout pairs
// (KCONTIG, KCONTIG), (KCONTIG, MNCONTIG): one translation unit per pair group so the
// family's many template instances compile in parallel.
#include "gemm_mfma16_kernel.h"

namespace mdemi {

KernelFn16 m16_pick_part0(int al, int bl, int aop, int bop, int np, int v) {
  if (al == MDEMI_L_KCONTIG && bl == MDEMI_L_KCONTIG) return m16_ops<MDEMI_L_KCONTIG, MDEMI_L_KCONTIG>(aop, bop, np, v);
  if (al == MDEMI_L_KCONTIG && bl == MDEMI_L_MNCONTIG) return m16_ops<MDEMI_L_KCONTIG, MDEMI_L_MNCONTIG>(aop, bop, np, v);
  return nullptr;
}

}  // namespace mdemi
