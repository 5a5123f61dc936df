// 16-bit-operand MFMA GEMM family on gfx950: v_mfma_f32_32x32x16_bf16
// (32 cycles per 32x32x16 block = 16x the v_mfma_f32_32x32x2_f32 rate), fp32
// accumulate, operands fetched as fp32 by the shared loaders (gemm_core.h) and
// split into NP bf16 planes on their way into LDS.
//
//   NP = 1  "bf16":  a = bf16(a).  torch.autocast's matmul numerics (BASELINE
//           configs[4], mixed precision).
//   NP = 3  "f32e":  a = a_hi + a_mid + a_lo exactly (each plane the RNE bf16 of
//           the remainder of the previous ones; 3 x 8 significant bits cover the
//           24 of an fp32), and
//             a.b ~= hi.hi + hi.mid + mid.hi + hi.lo + lo.hi + mid.mid
//           on six MFMAs.  Every bf16 x bf16 product is exact in the fp32
//           accumulator; the dropped terms (mid.lo, lo.mid, lo.lo) are below
//           2^-26 |a||b|, under one fp32 rounding of the product (2^-24).  So
//           this is an fp32 GEMM -- the error of the exact-product fp32 MFMA
//           kernel (gemm_f32.hip) -- at 6 x 32 instead of 8 x 64 MFMA cycles per
//           32x32x16 block: 2.67x the fp32 matrix peak (417 vs 157 TFLOP/s).
//
// Tiling: 128x128 block tile, BK = 32, 256 threads = 4 waves in 2x2, each wave
// 64x64 = 2x2 32x32 accumulators (the C layout, epilogue and split-K of
// gemm_f32.hip).  LDS images are [row][k] bf16 per plane (B as [col][k]), pitch
// 40 elements, with the 16-byte k-chunks of a row XOR-swizzled by
// swz(row): a lane's MFMA fragment (8 consecutive k of one row) is one
// ds_read_b128, conflict-free; the k-contiguous staging stores (ds_write_b64 of
// 4 k) and the transposed m/n-contiguous ones are 2-way (tools/lds_banks.py).
// m/n-contiguous sources (dgrad weights, wgrad operands) are loaded as 4 consecutive
// k rows x 4 columns per thread (Loader<..., KC = true>) and transposed in
// registers, so every store is a packed ds_write_b64 of 4 k.
#include "gemm_core.h"

namespace mdemi {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));

constexpr int M16_BK = 32;
constexpr int M16_PB = M16_BK + 8;            // image pitch (bf16 elements): 80 B
constexpr int M16_PLANE = GBM * M16_PB;       // bf16 elements per plane image

// 16-byte chunk swizzle of row `row` (chunks 0..3 of a 32-k row)
__device__ __forceinline__ int m16_swz(int row) {
  return ((((row >> 2) ^ (row >> 3) ^ (row >> 4)) & 1) << 1) | ((row >> 5) & 1);
}
// element offset of 8-byte half `half` of k-chunk `ch` of row `row`
__device__ __forceinline__ int m16_off(int row, int ch, int half) {
  return row * M16_PB + 8 * (ch ^ m16_swz(row)) + 4 * half;
}

// Split 4 fp32 values into NP packed bf16x4 planes (RNE each; the remainder of
// a value minus its bf16 rounding is exact in fp32).
template <int NP>
__device__ __forceinline__ void m16_split(float4 v, uint2 (&out)[NP]) {
  float2_t x01 = {v.x, v.y}, x23 = {v.z, v.w};
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const bf16x2_t h01 = __builtin_convertvector(x01, bf16x2_t);
    const bf16x2_t h23 = __builtin_convertvector(x23, bf16x2_t);
    out[p].x = __builtin_bit_cast(uint32_t, h01);
    out[p].y = __builtin_bit_cast(uint32_t, h23);
    if (p + 1 < NP) {
      x01 -= __builtin_convertvector(h01, float2_t);
      x23 -= __builtin_convertvector(h23, float2_t);
    }
  }
}

// Stage one operand tile (this thread's NQ = 4 float4) into the NP plane images.
template <int IMG, int NP>
__device__ __forceinline__ void m16_store(__bf16* img, int t, const float4 (&r)[M16_BK / 8]) {
  if constexpr (IMG == IMG_KR) {
    // KC loader: r[q] = columns 4*(t&31) .. +3 at k = 4*(t>>5) + q
    const int c4 = t & 31, kg = t >> 5;
    const float4 col[4] = {make_float4(r[0].x, r[1].x, r[2].x, r[3].x), make_float4(r[0].y, r[1].y, r[2].y, r[3].y),
                           make_float4(r[0].z, r[1].z, r[2].z, r[3].z), make_float4(r[0].w, r[1].w, r[2].w, r[3].w)};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint2 s[NP];
      m16_split<NP>(col[i], s);
      const int o = m16_off(4 * c4 + i, kg >> 1, kg & 1);
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(img + p * M16_PLANE + o) = s[p];
    }
  } else {
    // row t/8 + 32q, k-quad t%8
#pragma unroll
    for (int q = 0; q < M16_BK / 8; ++q) {
      uint2 s[NP];
      m16_split<NP>(r[q], s);
      const int kq = t & 7;
      const int o = m16_off((t >> 3) + 32 * q, kq >> 1, kq & 1);
#pragma unroll
      for (int p = 0; p < NP; ++p) *reinterpret_cast<uint2*>(img + p * M16_PLANE + o) = s[p];
    }
  }
}

#define MDEMI_MFMA16(A, B, C) C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, C, 0, 0, 0)

template <int AL, int BL, int AOP, int BOP, int NP, int NBUF>
__global__ __launch_bounds__(GTHREADS) void gemm_m16_kernel(GemmParams p) {
  constexpr int BK = M16_BK, NQ = BK / 8;
  using LA = Loader<AL, AOP, true, BK, false, true>;
  using LB = Loader<BL, BOP, false, BK, false, true>;
  constexpr int OPND = NP * M16_PLANE;  // one operand's images
  constexpr int BUFE = 2 * OPND;        // A + B
  static_assert(NBUF == 1 || NBUF == 2, "NBUF");
  __shared__ __attribute__((aligned(16))) __bf16 smem[NBUF * BUFE];

  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntiles = p.tiles_m * p.tiles_n;
  const int zb = blockIdx.x / ntiles;
  int tm, tn;
  tile_of(p, blockIdx.x % ntiles, ntiles, tm, tn);
  const int b = zb / p.split, sidx = zb % p.split;
  const int bm = tm * GBM, bn = tn * GBN;

  LA la;
  LB lb;
  la.init(p.A + (int64_t)b * p.a_bs, p.lda, p.M, p.K, p.a_vec, bm, t, p);
  lb.init(p.B + (int64_t)b * p.b_bs, p.ldb, p.N, p.K, p.b_vec, bn, t, p);

  const int ktiles_total = (p.K + BK - 1) / BK;
  const int kt_begin = sidx * p.ktile_per_split;
  const int kt_end = min(ktiles_total, kt_begin + p.ktile_per_split);

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  float4 ra[NQ], rb[NQ];
  constexpr bool CAN_RSUM = AL == MDEMI_L_MNCONTIG;
  const bool do_rsum = CAN_RSUM && p.rowsum != nullptr && tn == 0;
  float4 rsum = make_float4(0.f, 0.f, 0.f, 0.f);
  auto acc_rsum = [&]() {  // fp32 row sums of the unsplit A (bias gradient)
    if (CAN_RSUM && do_rsum) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        rsum.x += ra[q].x; rsum.y += ra[q].y; rsum.z += ra[q].z; rsum.w += ra[q].w;
      }
    }
  };
  const int l31 = lane & 31, h = lane >> 5;
  // fragment rows of this wave and their (swizzled) row bases
  int fa[2], fb[2], sa[2], sb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r_a = wm * 64 + 32 * i + l31, r_b = wn * 64 + 32 * i + l31;
    fa[i] = r_a * M16_PB; sa[i] = m16_swz(r_a);
    fb[i] = r_b * M16_PB; sb[i] = m16_swz(r_b);
  }

  auto stage = [&](__bf16* dst) {
    m16_store<LA::IMG, NP>(dst, t, ra);
    m16_store<LB::IMG, NP>(dst + OPND, t, rb);
    acc_rsum();
  };
  auto compute = [&](const __bf16* a_s) {
    const __bf16* b_s = a_s + OPND;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int ch = 2 * kk + h;
      bf16x8_t fA[2][NP], fB[2][NP];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          fA[i][q] = *reinterpret_cast<const bf16x8_t*>(a_s + q * M16_PLANE + fa[i] + 8 * (ch ^ sa[i]));
          fB[i][q] = *reinterpret_cast<const bf16x8_t*>(b_s + q * M16_PLANE + fb[i] + 8 * (ch ^ sb[i]));
        }
#pragma unroll
      for (int im = 0; im < 2; ++im)
#pragma unroll
        for (int in = 0; in < 2; ++in) {
          if constexpr (NP == 3) {  // small terms first, hi.hi last
            MDEMI_MFMA16(fA[im][1], fB[in][1], acc[im][in]);
            MDEMI_MFMA16(fA[im][2], fB[in][0], acc[im][in]);
            MDEMI_MFMA16(fA[im][0], fB[in][2], acc[im][in]);
            MDEMI_MFMA16(fA[im][1], fB[in][0], acc[im][in]);
            MDEMI_MFMA16(fA[im][0], fB[in][1], acc[im][in]);
          }
          MDEMI_MFMA16(fA[im][0], fB[in][0], acc[im][in]);
        }
    }
  };

  if (kt_begin < kt_end) {
    la.load(kt_begin * BK, ra);
    lb.load(kt_begin * BK, rb);
    stage(smem);
    __syncthreads();
  }
  int cur = 0;
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    if (more) {  // the next tile's loads land under this tile's MFMAs
      la.load((kt + 1) * BK, ra);
      lb.load((kt + 1) * BK, rb);
    }
    compute(smem + cur * BUFE);
    if (more) {
      if (NBUF == 1) __syncthreads();  // every wave done reading before the overwrite
      stage(smem + (NBUF == 1 ? 0 : (cur ^ 1)) * BUFE);
    }
    __syncthreads();
    if (NBUF == 2) cur ^= 1;
  }
  if (CAN_RSUM && do_rsum) {  // reduce the 8 k-row groups (t >> 5) through LDS
    float4* red = reinterpret_cast<float4*>(smem);
    red[t] = rsum;
    __syncthreads();
    if (t < 32) {
      float4 s4 = red[t];
#pragma unroll
      for (int g = 1; g < 8; ++g) {
        const float4 o = red[t + 32 * g];
        s4.x += o.x; s4.y += o.y; s4.z += o.z; s4.w += o.w;
      }
      float* dst = p.rowsum + (p.split > 1 ? (int64_t)sidx * p.M : 0);
      const int i = bm + 4 * t;
      if (i + 0 < p.M) dst[i + 0] = s4.x;
      if (i + 1 < p.M) dst[i + 1] = s4.y;
      if (i + 2 < p.M) dst[i + 2] = s4.z;
      if (i + 3 < p.M) dst[i + 3] = s4.w;
    }
  }
#include "gemm_epilogue.inc"
}
#undef MDEMI_MFMA16

using KernelFn16 = void (*)(GemmParams);

template <int AL, int BL, int AOP, int BOP>
static KernelFn16 m16_variant(int np, int v) {
  if (np == 3) return v == 1 ? gemm_m16_kernel<AL, BL, AOP, BOP, 3, 1> : gemm_m16_kernel<AL, BL, AOP, BOP, 3, 2>;
  return v == 1 ? gemm_m16_kernel<AL, BL, AOP, BOP, 1, 1> : gemm_m16_kernel<AL, BL, AOP, BOP, 1, 2>;
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

// Kernel of the 16-bit family for layouts (al, bl), load ops (aop, bop), NP
// planes (1: bf16, 3: split fp32) and variant v (0: two LDS buffers, 1: one).
void (*pick_kernel_m16(int al, int bl, int aop, int bop, int np, int v))(GemmParams) {
#define MDEMI_PICK(X, Y) \
  if (al == X && bl == Y) return m16_ops<X, Y>(aop, bop, np, v);
  MDEMI_PICK(MDEMI_L_KCONTIG, MDEMI_L_KCONTIG)
  MDEMI_PICK(MDEMI_L_KCONTIG, MDEMI_L_MNCONTIG)
  MDEMI_PICK(MDEMI_L_MNCONTIG, MDEMI_L_KCONTIG)
  MDEMI_PICK(MDEMI_L_MNCONTIG, MDEMI_L_MNCONTIG)
  MDEMI_PICK(MDEMI_L_CONV, MDEMI_L_KCONTIG)
  MDEMI_PICK(MDEMI_L_CONV, MDEMI_L_MNCONTIG)
  MDEMI_PICK(MDEMI_L_MNCONTIG, MDEMI_L_CONV)
  MDEMI_PICK(MDEMI_L_KCONTIG, MDEMI_L_CONV)
#undef MDEMI_PICK
  return nullptr;
}

}  // namespace mdemi
