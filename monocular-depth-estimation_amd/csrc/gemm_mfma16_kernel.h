// 16-bit-operand MFMA GEMM family on gfx950 (kernel template; instantiated per layout
// pair in gemm_m16_inst{0..3}.hip so the family compiles in parallel): v_mfma_f32_32x32x16_bf16
// (32 cycles per 32x32x16 block = 16x the v_mfma_f32_32x32x2_f32 rate), fp32
// accumulate.  Operands are fetched as fp32 by the shared loaders (gemm_core.h),
// staged in LDS as fp32 and split into NP bf16 planes as each wave reads its
// MFMA fragments.
//
//   NP = 1  "bf16":  a = bf16(a).  torch.autocast's matmul numerics (BASELINE
//           configs[4], mixed precision).
//   NP = 3  "f32e":  a = a_hi + a_mid + a_lo exactly (each plane the RNE bf16 of
//           the remainder of the previous ones; 3 x 8 significant bits cover the
//           24 of an fp32), and
//             a.b ~= hi.hi + hi.mid + mid.hi + hi.lo + lo.hi + mid.mid
//           on six MFMAs (the dropped mid.lo, lo.mid, lo.lo are below 2^-24 |a||b|),
//           at 6 x 32 instead of 8 x 64 MFMA cycles per 32x32x16 block: 2.67x the
//           fp32 matrix peak (417 vs 157 TFLOP/s).  Not bit-for-bit the accuracy of
//           the exact-product fp32 MFMA (gemm_f32.hip): on heavily cancelling sums
//           (a LayerNorm-bias gradient over 26,752 tokens at KITTI 352x1216) its
//           error is ~200x larger, and an eight-product form (dropping only lo.lo,
//           2^-32) measured the same error -- the difference comes from the bf16
//           MFMA's accumulation, not from the dropped planes
//           (profiles/round2/fp32e_parity_tests.txt).  Hence an opt-in precision.
//
// Tiling: 128x128 block tile, BK = 32, 256 threads = 4 waves in 2x2, each wave
// 64x64 = 2x2 32x32 accumulators (the C layout, epilogue and split-K of
// gemm_f32.hip).  m/n-contiguous sources (dgrad weights, wgrad operands) are
// loaded as 4 consecutive k rows x 4 columns per thread (Loader<..., KC = true>)
// and transposed in registers, so every LDS store runs along k.
//
// LDS image per operand: [row][k] fp32, pitch 32 floats (no pad), 16-B k-chunks
// XOR-swizzled by f32_swz(row) = ((row >> 1) ^ (row >> 4)) & 7: every fragment
// read (ds_read_b128) and every staging store (ds_write_b128, from a k- or an
// m/n-contiguous source) is conflict-free (tools/lds_banks.py).  Splitting at
// read time moves 4 B of LDS per element each way instead of the 6 of three
// staged bf16 planes (the LDS write rate, ~80 B/clk/CU, would otherwise take
// most of the MFMA time), and a double-buffered A+B tile pair is 64 KiB, so two
// workgroups share a CU and one's staging overlaps the other's MFMAs.
#pragma once
#include "gemm_core.h"

namespace mdemi {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));

constexpr int M16_BK = 32;
// ---- fp32 images; the bf16 planes are formed at fragment-read time ----
constexpr int F32_PITCH = M16_BK;  // floats per image row
__device__ __forceinline__ int f32_swz(int row) { return ((row >> 1) ^ (row >> 4)) & 7; }

template <int IMG>
__device__ __forceinline__ void f32_store(float* img, int t, const float4 (&r)[M16_BK / 8]) {
  if constexpr (IMG == IMG_KR) {  // KC loader: r[q] = columns 4*(t&31)..+3 at k = 4*(t>>5) + q
    const int c4 = t & 31, kg = t >> 5;
    const float4 col[4] = {make_float4(r[0].x, r[1].x, r[2].x, r[3].x), make_float4(r[0].y, r[1].y, r[2].y, r[3].y),
                           make_float4(r[0].z, r[1].z, r[2].z, r[3].z), make_float4(r[0].w, r[1].w, r[2].w, r[3].w)};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * c4 + i;
      *reinterpret_cast<float4*>(img + row * F32_PITCH + 4 * (kg ^ f32_swz(row))) = col[i];
    }
  } else {  // row t/8 + 32q, k-chunk t%8
#pragma unroll
    for (int q = 0; q < M16_BK / 8; ++q) {
      const int row = (t >> 3) + 32 * q;
      *reinterpret_cast<float4*>(img + row * F32_PITCH + 4 * ((t & 7) ^ f32_swz(row))) = r[q];
    }
  }
}

// ---- bf16 images (variants 3, 4; NP = 1): operands rounded once, as they are staged ----
// [row][32 k] bf16, 64 B per row, 16-B chunks (8 k) permuted by chunk ^ ((row >> 2) & 3):
// the fragment reads (ds_read_b128, 8 k of one row per lane) are conflict free.
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
constexpr int BF_ROW = M16_BK * 2;  // bytes per image row
__device__ __forceinline__ int bf_swz(int row) { return (row >> 2) & 3; }
__device__ __forceinline__ uint2 pack_bf16x4(float a, float b, float c, float d) {
  const bf16x2_t lo = __builtin_convertvector((float2_t){a, b}, bf16x2_t);
  const bf16x2_t hi = __builtin_convertvector((float2_t){c, d}, bf16x2_t);
  const bf16x4_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3);
  return *reinterpret_cast<const uint2*>(&v);
}
// 4 consecutive k (quad kq = 0..7 of the 32) of image row `row`, rounded to bf16, as 8 B
__device__ __forceinline__ void bf_put(char* img, int row, int kq, uint2 v) {
  *reinterpret_cast<uint2*>(img + row * BF_ROW + (((kq >> 1) ^ bf_swz(row)) << 4) + ((kq & 1) << 3)) = v;
}
template <int IMG>
__device__ __forceinline__ void bf16_store(char* img, int t, const float4 (&r)[M16_BK / 8]) {
  if constexpr (IMG == IMG_KR) {  // KC loader: r[q] = columns 4*(t&31)..+3 at k = 4*(t>>5) + q
    const int c4 = t & 31, kq = t >> 5;
    bf_put(img, 4 * c4 + 0, kq, pack_bf16x4(r[0].x, r[1].x, r[2].x, r[3].x));
    bf_put(img, 4 * c4 + 1, kq, pack_bf16x4(r[0].y, r[1].y, r[2].y, r[3].y));
    bf_put(img, 4 * c4 + 2, kq, pack_bf16x4(r[0].z, r[1].z, r[2].z, r[3].z));
    bf_put(img, 4 * c4 + 3, kq, pack_bf16x4(r[0].w, r[1].w, r[2].w, r[3].w));
  } else {  // row t/8 + 32q, k quad t%8
#pragma unroll
    for (int q = 0; q < M16_BK / 8; ++q)
      bf_put(img, (t >> 3) + 32 * q, t & 7, pack_bf16x4(r[q].x, r[q].y, r[q].z, r[q].w));
  }
}
// MFMA k-step kk's fragment (k = 16 kk + 8 h .. +7) of image row `row`
__device__ __forceinline__ bf16x8_t bf_frag(const char* img, int row, int kk, int h) {
  return *reinterpret_cast<const bf16x8_t*>(img + row * BF_ROW + (((2 * kk + h) ^ bf_swz(row)) << 4));
}

// 8 fp32 (k .. k+7 of one row) -> NP bf16x8 operand fragments: out[0] = RNE bf16 of the
// values, out[p] = RNE bf16 of what the planes before it leave (exact fp32 remainders)
template <int NP>
__device__ __forceinline__ void split8(const float4& u, const float4& v, bf16x8_t (&out)[NP]) {
  float2_t x[4] = {{u.x, u.y}, {u.z, u.w}, {v.x, v.y}, {v.z, v.w}};
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    bf16x2_t h[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      h[i] = __builtin_convertvector(x[i], bf16x2_t);
      if (p + 1 < NP) x[i] -= __builtin_convertvector(h[i], float2_t);
    }
    out[p] = __builtin_shufflevector(__builtin_shufflevector(h[0], h[1], 0, 1, 2, 3),
                                     __builtin_shufflevector(h[2], h[3], 0, 1, 2, 3), 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

#define MDEMI_MFMA16(A, B, C) C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, C, 0, 0, 0)

// BMT: block tile rows (128: 2x2 waves of 64x64; 256: 2x2 waves of 128x64, A staged
// as two 128-row images).  The block tile is 128 columns wide.
// BFL: operands rounded to bf16 as they are staged (bf16 LDS images, half the LDS bytes and
// one conversion per element instead of one per reading wave); NP = 1 only.  Same bf16
// values in the same MFMA positions as the fp32-image form: bit-identical results.
template <int AL, int BL, int AOP, int BOP, int NP, int NBUF, int BMT, bool BFL = false>
__global__ __launch_bounds__(GTHREADS) void gemm_m16_kernel(GemmParams p) {
  static_assert(!BFL || NP == 1, "bf16 LDS images hold one plane");
  constexpr int BK = M16_BK, NQ = BK / 8;
  constexpr int NA = BMT / 128;     // 128-row A images per tile
  constexpr int IM = BMT / 64;      // 32-row accumulator blocks per wave along M
  constexpr int WTM = BMT / 2;      // wave tile rows
  using LA = Loader<AL, AOP, true, BK, false, true>;
  using LB = Loader<BL, BOP, false, BK, false, true>;
  constexpr int IMG_B = BFL ? GBM * BF_ROW : GBM * F32_PITCH * 4;  // bytes of one 128-row image
  constexpr int BUF_B = (NA + 1) * IMG_B;     // A images + the B image
  static_assert(NBUF == 1 || NBUF == 2, "NBUF");
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF_B];

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
  constexpr bool CAN_RSUM = AL == MDEMI_L_MNCONTIG;
  const bool do_rsum = CAN_RSUM && p.rowsum != nullptr && tn == 0;
  float4 rsum[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) rsum[a] = make_float4(0.f, 0.f, 0.f, 0.f);
  auto acc_rsum = [&]() {  // fp32 row sums of the unsplit A (bias gradient)
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
  // this wave's fragment rows: A rows (within image wm*WTM/128), B columns
  int rA[IM], rB[2];
#pragma unroll
  for (int i = 0; i < IM; ++i) rA[i] = (wm * WTM + 32 * i + l31) & 127;
#pragma unroll
  for (int i = 0; i < 2; ++i) rB[i] = wn * 64 + 32 * i + l31;
  const int aimg = (wm * WTM) >> 7;  // A image holding this wave's rows

  auto load = [&](int kt) {
#pragma unroll
    for (int a = 0; a < NA; ++a) la[a].load(kt * BK, ra[a]);
    lb.load(kt * BK, rb);
  };
  auto stage = [&](char* dst) {
    if constexpr (BFL) {
#pragma unroll
      for (int a = 0; a < NA; ++a) bf16_store<LA::IMG>(dst + a * IMG_B, t, ra[a]);
      bf16_store<LB::IMG>(dst + NA * IMG_B, t, rb);
    } else {
#pragma unroll
      for (int a = 0; a < NA; ++a) f32_store<LA::IMG>(reinterpret_cast<float*>(dst + a * IMG_B), t, ra[a]);
      f32_store<LB::IMG>(reinterpret_cast<float*>(dst + NA * IMG_B), t, rb);
    }
    acc_rsum();
  };
  auto compute = [&](const char* buf) {
    if constexpr (BFL) {
      const char* a_s = buf + aimg * IMG_B;
      const char* b_s = buf + NA * IMG_B;
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) {
        bf16x8_t A[IM], B[2];
#pragma unroll
        for (int i = 0; i < IM; ++i) A[i] = bf_frag(a_s, rA[i], kk, h);
#pragma unroll
        for (int i = 0; i < 2; ++i) B[i] = bf_frag(b_s, rB[i], kk, h);
#pragma unroll
        for (int im = 0; im < IM; ++im)
#pragma unroll
          for (int in = 0; in < 2; ++in) MDEMI_MFMA16(A[im], B[in], acc[im][in]);
      }
      return;
    }
    const float* a_s = reinterpret_cast<const float*>(buf + aimg * IMG_B);
    const float* b_s = reinterpret_cast<const float*>(buf + NA * IMG_B);
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      float4 fa[IM][2], fb[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = 4 * kk + 2 * h + j;
#pragma unroll
        for (int i = 0; i < IM; ++i)
          fa[i][j] = *reinterpret_cast<const float4*>(a_s + rA[i] * F32_PITCH + 4 * (c ^ f32_swz(rA[i])));
#pragma unroll
        for (int i = 0; i < 2; ++i)
          fb[i][j] = *reinterpret_cast<const float4*>(b_s + rB[i] * F32_PITCH + 4 * (c ^ f32_swz(rB[i])));
      }
      bf16x8_t A[IM][NP], B[2][NP];
#pragma unroll
      for (int i = 0; i < IM; ++i) {
#ifdef MDEMI_M16_ABLATE_SPLIT  // study: the NP-plane MFMA schedule with one conversion
        bf16x8_t a1[1];
        split8<1>(fa[i][0], fa[i][1], a1);
#pragma unroll
        for (int q = 0; q < NP; ++q) A[i][q] = a1[0];
#else
        split8<NP>(fa[i][0], fa[i][1], A[i]);
#endif
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) split8<NP>(fb[i][0], fb[i][1], B[i]);
#pragma unroll
      for (int im = 0; im < IM; ++im)
#pragma unroll
        for (int in = 0; in < 2; ++in) {
          if constexpr (NP == 3) {  // small terms first, hi.hi last
            MDEMI_MFMA16(A[im][1], B[in][1], acc[im][in]);
            MDEMI_MFMA16(A[im][2], B[in][0], acc[im][in]);
            MDEMI_MFMA16(A[im][0], B[in][2], acc[im][in]);
            MDEMI_MFMA16(A[im][1], B[in][0], acc[im][in]);
            MDEMI_MFMA16(A[im][0], B[in][1], acc[im][in]);
          }
          MDEMI_MFMA16(A[im][0], B[in][0], acc[im][in]);
        }
    }
  };

  if (kt_begin < kt_end) {
    load(kt_begin);
    stage(smem);
    __syncthreads();
  }
  int cur = 0;
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    if (more) load(kt + 1);  // the next tile's loads land under this tile's MFMAs
    compute(smem + cur * BUF_B);
    if (more) {
      if (NBUF == 1) __syncthreads();  // every wave done reading before the overwrite
      stage(smem + (NBUF == 1 ? 0 : (cur ^ 1)) * BUF_B);
    }
    __syncthreads();
    if (NBUF == 2) cur ^= 1;
  }
  if (CAN_RSUM && do_rsum) {  // reduce the 8 k-row groups (t >> 5) of each A half through LDS
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
#undef MDEMI_MFMA16

using KernelFn16 = void (*)(GemmParams);

// 16-bit family variants: 0 = 128-row tile, two LDS buffers; 1 = 128-row tile, one
// buffer (two workgroups per CU by LDS); 2 = 256-row tile, two buffers (96 KiB);
// 3 / 4 = bf16 LDS images (bf16 only), 128- / 256-row tile, two buffers (32 / 48 KiB).
// Every variant adds each output's products in the same order (bit-identical).
template <int AL, int BL, int AOP, int BOP>
static KernelFn16 m16_variant(int np, int v) {
  if (v >= 3) {  // bf16 LDS images (NP = 1): 3 = 128-row tile, 4 = 256-row tile, two buffers each
    if (np != 1) return nullptr;
    return v == 4 ? gemm_m16_kernel<AL, BL, AOP, BOP, 1, 2, 256, true> : gemm_m16_kernel<AL, BL, AOP, BOP, 1, 2, 128, true>;
  }
  if (np == 3) {
    if (v == 2) return gemm_m16_kernel<AL, BL, AOP, BOP, 3, 2, 256>;
    return v == 1 ? gemm_m16_kernel<AL, BL, AOP, BOP, 3, 1, 128> : gemm_m16_kernel<AL, BL, AOP, BOP, 3, 2, 128>;
  }
  if (v == 2) return gemm_m16_kernel<AL, BL, AOP, BOP, 1, 2, 256>;
  return v == 1 ? gemm_m16_kernel<AL, BL, AOP, BOP, 1, 1, 128> : gemm_m16_kernel<AL, BL, AOP, BOP, 1, 2, 128>;
}
template <int AL, int BL>
static KernelFn16 m16_ops(int aop, int bop, int np, int v) {
  if (aop == MDEMI_OP_NONE && bop == MDEMI_OP_NONE) return m16_variant<AL, BL, MDEMI_OP_NONE, MDEMI_OP_NONE>(np, v);
  if constexpr (AL == MDEMI_L_KCONTIG)
    if (aop == MDEMI_OP_GELU && bop == MDEMI_OP_NONE) return m16_variant<AL, BL, MDEMI_OP_GELU, MDEMI_OP_NONE>(np, v);
  if constexpr (BL == MDEMI_L_MNCONTIG)
    if (aop == MDEMI_OP_NONE && bop == MDEMI_OP_GELU) return m16_variant<AL, BL, MDEMI_OP_NONE, MDEMI_OP_GELU>(np, v);
  return nullptr;
}

}  // namespace mdemi
