// fp32 MFMA GEMM kernel template and its variant / load-op pickers (see gemm_f32.hip
// for the design); instantiated per layout pair in gemm_f32_inst{0..3}.hip so the
// family compiles in parallel.
#pragma once
#include "common.h"
#include "gemm_core.h"

namespace mdemi {

using KernelFn = void (*)(GemmParams);

// Pipelining variants (A/B-tested on the model's shapes, tools/gemm_bench.py):
//   BK    K depth per LDS tile (16 or 32)
//   NBUF  LDS buffers (2: write the next tile while others read this one)
//   PREF  register prefetch of the next tile before the MFMAs (issue early / write late)
//   BMT   block-tile rows: 128 (2x2 waves of 64x64) or 256 (2x2 waves of 128x64, A staged as
//         two 128-row images: twice the MFMAs per barrier and per B fragment)
// Variants 8..11 stage by DMA straight into LDS (gemm_glds_kernel.h).
template <int AL, int BL, int AOP, int BOP, int BK, int NBUF, bool PREF, bool TR, int OCC, int BMT = 128>
__global__ __launch_bounds__(GTHREADS) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void gemm_f32_kernel(GemmParams p) {
  using LA = Loader<AL, AOP, true, BK, TR>;
  using LB = Loader<BL, BOP, false, BK, TR>;
  constexpr int FA = Img<LA::IMG, BK>::floats, FB = Img<LB::IMG, BK>::floats;
  constexpr int NQ = BK / 8;
  constexpr int NA = BMT / 128;  // 128-row A images per tile
  constexpr int IM = BMT / 64;   // 32-row accumulator blocks per wave along M
  constexpr int WTM = BMT / 2;   // wave tile rows
  constexpr int FAT = NA * FA;   // floats of the A images
  static_assert(NBUF == 2 || NBUF == 1, "NBUF");
  static_assert(BK == 16 || BK == 32, "BK");
  static_assert(BMT == 128 || BMT == 256, "BMT");
  __shared__ __attribute__((aligned(16))) float smem[NBUF * (FAT + FB)];

  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const GemmJob job = job_of(p);
  const int b = job.b, sidx = job.sidx, tm = job.tm, tn = job.tn;
  const int bm = tm * BMT, bn = tn * GBN;

  LA la[NA];
  LB lb;
#pragma unroll
  for (int a = 0; a < NA; ++a)
    la[a].init(p.A + boff(p, b, p.a_bs, p.a_bs2), p.lda, p.M, p.K, p.a_vec, bm + 128 * a, t, p);
  lb.init(p.B + boff(p, b, p.b_bs, p.b_bs2), p.ldb, p.N, p.K, p.b_vec, bn, t, p);

  const int ktiles_total = (p.K + BK - 1) / BK;
  const int kt_begin = job.split ? sidx * p.ktile_per_split : 0;
  const int kt_end = job.split ? min(ktiles_total, kt_begin + p.ktile_per_split) : ktiles_total;

  floatx16 acc[IM][2];
#pragma unroll
  for (int a = 0; a < IM; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  float4 ra[NA][NQ], rb[NQ];
  // Row sums of an m-contiguous A (the bias gradient of a weight-gradient
  // GEMM, dW = dY^T X, db = dY^T 1) accumulated from the staged registers
  // by the tn == 0 column of workgroups: no second pass over dY.
  constexpr bool CAN_RSUM = AL == MDEMI_L_MNCONTIG;
  const bool do_rsum = CAN_RSUM && p.rowsum != nullptr && tn == 0;
  float4 rsum[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) rsum[a] = make_float4(0.f, 0.f, 0.f, 0.f);
  auto acc_rsum = [&]() {
    if (CAN_RSUM && do_rsum) {
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          rsum[a].x += ra[a][q].x; rsum[a].y += ra[a][q].y; rsum[a].z += ra[a][q].z; rsum[a].w += ra[a][q].w;
        }
    }
  };
  const int l31 = lane & 31, h = lane >> 5;
  int rA[IM];  // this wave's fragment rows within A image aimg
#pragma unroll
  for (int i = 0; i < IM; ++i) rA[i] = (wm * WTM + 32 * i + l31) & 127;
  const int aimg = (wm * WTM) >> 7;
  const int rb0 = wn * 64 + l31, rb1 = rb0 + 32;

#ifdef MDEMI_STUDY_NOLOAD  // study build: no global operand loads (LDS + MFMA + barrier ceiling)
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int q = 0; q < NQ; ++q) ra[a][q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int q = 0; q < NQ; ++q) rb[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  auto load = [&](int) {};
#else
  auto load = [&](int kt) {
#pragma unroll
    for (int a = 0; a < NA; ++a) la[a].load(kt * BK, ra[a]);
    lb.load(kt * BK, rb);
  };
#endif
  auto stage = [&](float* dst) {
#pragma unroll
    for (int a = 0; a < NA; ++a) LA::store(dst + a * FA, t, ra[a]);
    LB::store(dst + FAT, t, rb);
    acc_rsum();
  };

  if (PREF && kt_begin < kt_end) {
    load(kt_begin);
    stage(smem);
    __syncthreads();
  }

  int cur = 0;
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    if (!PREF) {  // plain: load, stage, barrier, compute (other workgroups overlap)
      load(kt);
      stage(smem);
      __syncthreads();
    } else if (more) {  // issue next tile's global loads early; they land under the MFMAs
      load(kt + 1);
    }
    const float* a_s = smem + cur * (FAT + FB) + aimg * FA;
    const float* b_s = smem + cur * (FAT + FB) + FAT;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      float4 fa[IM];
#pragma unroll
      for (int i = 0; i < IM; ++i) fa[i] = Img<LA::IMG, BK>::frag(a_s, rA[i], g, h);
      const float4 b0 = Img<LB::IMG, BK>::frag(b_s, rb0, g, h);
      const float4 b1 = Img<LB::IMG, BK>::frag(b_s, rb1, g, h);
#define MDEMI_STEP(X)                                                                        \
  _Pragma("unroll") for (int i = 0; i < IM; ++i) {                                           \
    acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].X, b0.X, acc[i][0], 0, 0, 0);     \
    acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].X, b1.X, acc[i][1], 0, 0, 0);     \
  }
      MDEMI_STEP(x) MDEMI_STEP(y) MDEMI_STEP(z) MDEMI_STEP(w)
#undef MDEMI_STEP
    }
#ifdef MDEMI_STUDY_NOSYNC  // study build: no restaging and no barrier (LDS reads + MFMA ceiling)
    if (true) {
    } else
#endif
    if (!PREF) {
      __syncthreads();
    } else {
      if (more) {
        if (NBUF == 1) __syncthreads();  // everyone done reading before overwrite
        stage(smem + (NBUF == 1 ? 0 : (cur ^ 1)) * (FAT + FB));
      }
      __syncthreads();
      if (NBUF == 2) cur ^= 1;
    }
  }
  if (CAN_RSUM && do_rsum) {  // reduce the 8 k-row groups (t >> 5) of each A image through LDS
    if (!PREF) __syncthreads();
    float4* red = reinterpret_cast<float4*>(smem);
#pragma unroll
    for (int a = 0; a < NA; ++a) red[a * 256 + t] = rsum[a];
    __syncthreads();
    if (t < 32 * NA) {
      const int a = t >> 5, tt = t & 31;
      float4 s4 = red[a * 256 + tt];
#pragma unroll
      for (int g = 1; g < 8; ++g) {
        const float4 o = red[a * 256 + tt + 32 * g];
        s4.x += o.x; s4.y += o.y; s4.z += o.z; s4.w += o.w;
      }
      store_rowsum4(p, sidx, bm + 128 * a + 4 * tt, s4);
    }
  }

#define EP_IM IM
#define EP_WTM WTM
#include "gemm_epilogue.inc"
}

template <int AL, int BL, int AOP, int BOP>
static KernelFn pick_variant(int v) {
  if (v >= 8) return nullptr;  // direct-to-LDS staging: gemm_glds_inst*.hip (gemm_f32.hip pick_kernel)
  switch (v) {
    case 1: return gemm_f32_kernel<AL, BL, AOP, BOP, 16, 2, true, false, 2>;
    case 2: return gemm_f32_kernel<AL, BL, AOP, BOP, 16, 2, true, true, 4>;
    case 3: return gemm_f32_kernel<AL, BL, AOP, BOP, 32, 2, true, true, 2>;
    case 4: return gemm_f32_kernel<AL, BL, AOP, BOP, 32, 1, true, true, 3>;
    case 5: return gemm_f32_kernel<AL, BL, AOP, BOP, 32, 2, true, false, 2>;
    case 6: return gemm_f32_kernel<AL, BL, AOP, BOP, 32, 1, true, true, 2, 256>;
    case 7: return gemm_f32_kernel<AL, BL, AOP, BOP, 16, 2, true, true, 2, 256>;
    default: return gemm_f32_kernel<AL, BL, AOP, BOP, 16, 2, true, true, 2>;
  }
}

template <int AL, int BL>
static KernelFn pick_ops(int aop, int bop, int v) {
  if (aop == MDEMI_OP_NONE && bop == MDEMI_OP_NONE) return pick_variant<AL, BL, MDEMI_OP_NONE, MDEMI_OP_NONE>(v);
  if constexpr (AL == MDEMI_L_KCONTIG)
    if (aop == MDEMI_OP_GELU && bop == MDEMI_OP_NONE)
      return pick_variant<AL, BL, MDEMI_OP_GELU, MDEMI_OP_NONE>(v);
  if constexpr (BL == MDEMI_L_MNCONTIG)
    if (aop == MDEMI_OP_NONE && bop == MDEMI_OP_GELU)
      return pick_variant<AL, BL, MDEMI_OP_NONE, MDEMI_OP_GELU>(v);
  return nullptr;
}

}  // namespace mdemi
