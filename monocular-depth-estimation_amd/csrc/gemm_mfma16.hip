// 16-bit-operand MFMA GEMM family: kernel selection over the per-layout-pair
// instantiation units (gemm_m16_inst*.hip); the kernel is in gemm_mfma16_kernel.h.
#include "gemm_core.h"

namespace mdemi {

using KernelFn16 = void (*)(GemmParams);
KernelFn16 m16_pick_part0(int al, int bl, int aop, int bop, int np, int v);
KernelFn16 m16_pick_part1(int al, int bl, int aop, int bop, int np, int v);
KernelFn16 m16_pick_part2(int al, int bl, int aop, int bop, int np, int v);
KernelFn16 m16_pick_part3(int al, int bl, int aop, int bop, int np, int v);

// Kernel of the 16-bit family for layouts (al, bl), load ops (aop, bop), NP
// planes (1: bf16, 3: split fp32) and variant v (see m16_variant).
void (*pick_kernel_m16(int al, int bl, int aop, int bop, int np, int v))(GemmParams) {
  if (KernelFn16 f = m16_pick_part0(al, bl, aop, bop, np, v)) return f;
  if (KernelFn16 f = m16_pick_part1(al, bl, aop, bop, np, v)) return f;
  if (KernelFn16 f = m16_pick_part2(al, bl, aop, bop, np, v)) return f;
  return m16_pick_part3(al, bl, aop, bop, np, v);
}

}  // namespace mdemi
