// bf16-operand GEMM on gfx950: A and B are bf16 tensors in HBM (the bf16 storage path of
// precision "bf16", BASELINE configs[4]); v_mfma_f32_32x32x16_bf16 with fp32 accumulation;
// operands DMA'd global -> LDS (`buffer_load_dwordx4 ... lds`, 16 B = 8 bf16 per lane), no
// VGPR staging and no conversion in the K loop.  The products, their k order and the split-K
// boundaries are those of the bf16 m16 family (gemm_mfma16_kernel.h, variants 3/4: operands
// rounded to bf16 as they are staged), so for operands that are the RNE bf16 of the fp32
// tensors the m16 family reads, every output is bit-identical -- storing an activation in
// bf16 instead of fp32 changes no result, only the bytes moved.
//
// Why: the m16 family streams fp32 operands through VGPRs (8 global loads, 16 conversions
// and 8 LDS stores per thread per 128x128x32 tile against 8 MFMAs of 32 cycles per wave),
// which holds it near 0.06 of the bf16 MFMA peak.  Here a wave issues one
// DMA instruction per KiB of tile and nothing else, and operand bytes are halved.
//
// LDS images (one per 128 rows / columns of a stage; every swizzle is applied to the
// per-lane GLOBAL address, since a DMA lands lane-linearly):
//   k-contiguous source (and implicit-im2col A): [row][32 k] bf16, 64-B rows, 16-B chunk c
//     (8 k) at slot c ^ ((row >> 2) & 3); a lane's MFMA fragment (8 consecutive k of one row)
//     is one conflict-free ds_read_b128 (the m16 BFL image).
//   m/n-contiguous source (and implicit-im2col B): [32 k][128 columns] bf16, 256-B rows,
//     16-B chunk c (8 columns) at slot c ^ (((k & 3) << 2) | ((k >> 2) & 3)); a fragment (8
//     consecutive k of one column) is two ds_read_b64_tr_b16 (4 k each, the hardware
//     transpose), conflict-free with this swizzle (cdna_hip_programming.md T10 (b);
//     tools/lds_banks.py).
// Pipeline: two LDS stages as separate __shared__ objects, loop unrolled by two; the DMA of
// k tile kt+1 is issued before tile kt's MFMAs and retired by `s_waitcnt vmcnt(0)` + one
// barrier after them.
#pragma once
#include <type_traits>

#include "common.h"
#include "gemm_core.h"

namespace mdemi {

typedef __bf16 b16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void b16_lds_void_t;
typedef __attribute__((address_space(3))) s16x4_t b16_lds_s4_t;

constexpr int B16_BK = 32;         // k per tile (the split-K chunk)
constexpr int B16_IMG = 128 * 64;  // bytes of one image: 128 rows x 64 B, or 32 k x 256 B

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc16(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, BUF_RECORDS, 0x00020000);
}
__device__ __forceinline__ void b16_dma(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (b16_lds_void_t*)lds, 16, voff, 0, 0, 0);
}
__device__ __forceinline__ int kc_swz(int row) { return (row >> 2) & 3; }
__device__ __forceinline__ int mn_swz(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }

// 8 consecutive k (16 kk + 8 h ..) of row r of a [row][32 k] image
__device__ __forceinline__ b16x8_t kc_frag(const char* img, int r, int kk, int h) {
  return *reinterpret_cast<const b16x8_t*>(img + r * 64 + (((2 * kk + h) ^ kc_swz(r)) << 4));
}
// 8 consecutive k of column cb + (lane & 31) of a [32 k][128 col] image: two transposed reads.
// Lane 4q+p of 16-lane group g supplies row k0 + q (k0 = 16 kk + 8 (g >> 1), then + 4),
// columns col0 + 4p .. +3 (col0 = cb + 16 (g & 1)); lane i of the group receives column
// col0 + i, row q in element q.
__device__ __forceinline__ b16x8_t mn_frag(const char* img, int cb, int kk, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = cb + 16 * (g & 1) + 4 * p;
  const int k0 = 16 * kk + 8 * (g >> 1) + q;
  const int ch = col >> 3, hb = (col >> 2) & 1;
  const char* a0 = img + k0 * 256 + ((ch ^ mn_swz(k0)) << 4) + 8 * hb;
  const char* a1 = img + (k0 + 4) * 256 + ((ch ^ mn_swz(k0 + 4)) << 4) + 8 * hb;
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((b16_lds_s4_t*)a0);
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((b16_lds_s4_t*)a1);
  const s16x4_t v[2] = {lo, hi};
  return *reinterpret_cast<const b16x8_t*>(v);
}

// ---- loaders: one 128-row (or 128-column) image per call; wave w issues instructions
// q = 2w, 2w + 1 (8 per image, 1 KiB each) ----

// dense k-contiguous [rows][K] (k stride 1, row stride ld): instruction q covers rows
// 16q .. 16q+15, lane j -> row 16q + j/4, slot j%4
struct B16LoadKC {
  const char* base; int K;
  int voff[2], kch[2];
  __device__ void init(const void* p, int64_t ld, int rows, int K_, int r0, int wid, int lane, const GemmParams&) {
    base = reinterpret_cast<const char*>(p) + (int64_t)r0 * ld * 2; K = K_;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 16 * (2 * wid + i) + (lane >> 2);
      const int ch = (lane & 3) ^ kc_swz(row);
      kch[i] = ch;
      voff[i] = r0 + row < rows ? (int)(((int64_t)row * ld + 8 * ch) * 2) : BUF_OOB;
    }
  }
  __device__ void issue(int k0, char* img, int wid) const {
    const auto rs = make_rsrc16(base + (int64_t)k0 * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) b16_dma(rs, img + (2 * wid + i) * 1024, k0 + 8 * kch[i] < K ? voff[i] : BUF_OOB);
  }
};

// dense m/n-contiguous [K][cols] (column stride 1, k stride ld): instruction q covers k rows
// 4q .. 4q+3, lane j -> k row 4q + j/16, slot j%16
struct B16LoadMN {
  const char* base; int64_t ld; int K;
  int voff[2], kr[2];
  __device__ void init(const void* p, int64_t ld_, int cols, int K_, int c0, int wid, int lane, const GemmParams&) {
    base = reinterpret_cast<const char*>(p) + (int64_t)c0 * 2; ld = ld_; K = K_;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = 4 * (2 * wid + i) + (lane >> 4);
      const int ch = (lane & 15) ^ mn_swz(k);
      kr[i] = k;
      voff[i] = c0 + 8 * ch < cols ? (int)(((int64_t)k * ld + 8 * ch) * 2) : BUF_OOB;
    }
  }
  __device__ void issue(int k0, char* img, int wid) const {
    const auto rs = make_rsrc16(base + (int64_t)k0 * ld * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) b16_dma(rs, img + (2 * wid + i) * 1024, k0 + kr[i] < K && voff[i] != BUF_OOB ? voff[i] : BUF_OOB);
  }
};

// implicit im2col of an NHWC bf16 activation, operand A (row = output pixel, k = (ky,kx,c)):
// the k-contiguous image, each lane's 8 k one tap's 8 consecutive channels (C % 8 == 0)
struct B16LoadConvA {
  const char* base; mdemi_conv_geom g; FastDiv fc, fkw; int K;
  int n[2], iy0[2], ix0[2], kch[2]; bool valid[2];
  __device__ void init(const void* p, int64_t, int rows, int K_, int r0, int wid, int lane, const GemmParams& P) {
    base = reinterpret_cast<const char*>(p); g = P.cv; fc = P.fd_c; fkw = P.fd_kw; K = K_;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 16 * (2 * wid + i) + (lane >> 2);
      kch[i] = (lane & 3) ^ kc_swz(row);
      const int pix = r0 + row;
      valid[i] = pix < rows;
      const int ii = valid[i] ? pix : 0;
      const int tmp = fdiv(ii, P.fd_ow), ox = ii - tmp * g.ow;
      const int nn = fdiv(tmp, P.fd_oh), oy = tmp - nn * g.oh;
      n[i] = nn;
      iy0[i] = oy * g.stride - g.pad;
      ix0[i] = ox * g.stride - g.pad;
    }
  }
  __device__ void issue(int k0, char* img, int wid) const {
    const auto rs = make_rsrc16(base);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = k0 + 8 * kch[i];
      bool ok = valid[i] && k < K;
      const int kk = ok ? k : 0;
      const int tap = fdiv(kk, fc), c = kk - tap * g.c;
      const int ky = fdiv(tap, fkw), kx = tap - ky * g.kw;
      int iy = iy0[i] + ky, ix = ix0[i] + kx;
      if (g.pad_mode == MDEMI_PAD_REPLICATE) {
        iy = min(max(iy, 0), g.h - 1); ix = min(max(ix, 0), g.w - 1);
      } else {
        ok = ok && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
      }
      const int off = (int)(((((int64_t)n[i] * g.h + iy) * g.w + ix) * g.c + c) * 2);
      b16_dma(rs, img + (2 * wid + i) * 1024, ok ? off : BUF_OOB);
    }
  }
};

// implicit im2col, operand B (weight gradients): B(k = output pixel, j = (ky,kx,c)), the
// m/n-contiguous image; a lane's (tap, channel) is fixed, its pixel advances with k
struct B16LoadConvB {
  const char* base; mdemi_conv_geom g; FastDiv fow, foh; int K;
  int kr[2], ky[2], kx[2], c[2]; bool jvalid[2];
  __device__ void init(const void* p, int64_t, int cols, int K_, int c0, int wid, int lane, const GemmParams& P) {
    base = reinterpret_cast<const char*>(p); g = P.cv; fow = P.fd_ow; foh = P.fd_oh; K = K_;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = 4 * (2 * wid + i) + (lane >> 4);
      kr[i] = k;
      const int j = c0 + 8 * ((lane & 15) ^ mn_swz(k));
      jvalid[i] = j < cols;
      const int jj = jvalid[i] ? j : 0;
      const int tap = fdiv(jj, P.fd_c);
      c[i] = jj - tap * g.c;
      ky[i] = fdiv(tap, P.fd_kw);
      kx[i] = tap - ky[i] * g.kw;
    }
  }
  __device__ void issue(int k0, char* img, int wid) const {
    const auto rs = make_rsrc16(base);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = k0 + kr[i];
      bool ok = jvalid[i] && k < K;
      const int kk = ok ? k : 0;
      const int tmp = fdiv(kk, fow), ox = kk - tmp * g.ow;
      const int nn = fdiv(tmp, foh), oy = tmp - nn * g.oh;
      int iy = oy * g.stride - g.pad + ky[i], ix = ox * g.stride - g.pad + kx[i];
      if (g.pad_mode == MDEMI_PAD_REPLICATE) {
        iy = min(max(iy, 0), g.h - 1); ix = min(max(ix, 0), g.w - 1);
      } else {
        ok = ok && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
      }
      const int off = (int)(((((int64_t)nn * g.h + iy) * g.w + ix) * g.c + c[i]) * 2);
      b16_dma(rs, img + (2 * wid + i) * 1024, ok ? off : BUF_OOB);
    }
  }
};

template <int L, bool IS_A>
using B16Load = typename std::conditional<
    L == MDEMI_L_KCONTIG, B16LoadKC,
    typename std::conditional<L == MDEMI_L_MNCONTIG, B16LoadMN,
                              typename std::conditional<IS_A, B16LoadConvA, B16LoadConvB>::type>::type>::type;

// k-contiguous-image layouts (row fragments by ds_read_b128) vs transposed-image layouts
template <int L, bool IS_A>
struct B16RowImg {
  static constexpr bool v = L == MDEMI_L_KCONTIG || (L == MDEMI_L_CONV && IS_A);
};

// BMT: block-tile rows (128: 2x2 waves of 64x64; 256: 2x2 waves of 128x64, A as two
// 128-row images).  OCC: waves per SIMD the register budget targets.  KT2: K tiles per LDS
// stage (1, or 2 for 128-row tiles: 16 MFMAs per wave between barriers instead of 8, for the
// small GEMMs whose per-tile fixed cost dominates); the tiles still run in k order.
template <int AL, int BL, int BMT, int OCC, int KT2 = 1>
__global__ __launch_bounds__(GTHREADS) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void gemm_b16_kernel(
    GemmParams p) {
  constexpr int NA = BMT / 128, IM = BMT / 64, WTM = BMT / 2;
  static_assert(KT2 == 1 || (KT2 == 2 && NA == 1), "two K tiles per stage: 128-row tiles");
  constexpr int TILE = (NA + 1) * B16_IMG;  // one K tile's images
  constexpr int STAGE = KT2 * TILE;
  constexpr bool AROW = B16RowImg<AL, true>::v, BROW = B16RowImg<BL, false>::v;
  // stage 0 is `smem` (the epilogue's split-K hand-off flag reuses it after the loop)
  __shared__ __attribute__((aligned(16))) char smem[STAGE];
  __shared__ __attribute__((aligned(16))) char smem1[STAGE];

  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const GemmJob job = job_of(p);
  const int b = job.b, sidx = job.sidx, tm = job.tm, tn = job.tn;
  const int bm = tm * BMT, bn = tn * GBN;

  using LA = B16Load<AL, true>;
  using LB = B16Load<BL, false>;
  const char* A16 = reinterpret_cast<const char*>(p.A) + boff(p, b, p.a_bs, p.a_bs2) * 2;
  const char* B16 = reinterpret_cast<const char*>(p.B) + boff(p, b, p.b_bs, p.b_bs2) * 2;
  LA la[NA];
  LB lb;
#pragma unroll
  for (int a = 0; a < NA; ++a) la[a].init(A16, p.lda, p.M, p.K, bm + 128 * a, wid, lane, p);
  lb.init(B16, p.ldb, p.N, p.K, bn, wid, lane, p);

  const int ktiles_total = (p.K + B16_BK - 1) / B16_BK;
  const int kt_begin = job.split ? sidx * p.ktile_per_split : 0;
  const int kt_end = job.split ? min(ktiles_total, kt_begin + p.ktile_per_split) : ktiles_total;

  floatx16 acc[IM][2];
#pragma unroll
  for (int a = 0; a < IM; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  auto issue = [&](int kt, char* st) {
#pragma unroll
    for (int a = 0; a < NA; ++a) la[a].issue(kt * B16_BK, st + a * B16_IMG, wid);
    lb.issue(kt * B16_BK, st + NA * B16_IMG, wid);
  };

  const int l31 = lane & 31, h = lane >> 5;
  const int aimg = (wm * WTM) >> 7;
  auto fragA = [&](const char* a_s, int i, int kk) -> b16x8_t {
    const int r = (wm * WTM + 32 * i) & 127;
    if constexpr (AROW) return kc_frag(a_s, r + l31, kk, h);
    else return mn_frag(a_s, r, kk, lane);
  };
  auto fragB = [&](const char* b_s, int i, int kk) -> b16x8_t {
    const int r = wn * 64 + 32 * i;
    if constexpr (BROW) return kc_frag(b_s, r + l31, kk, h);
    else return mn_frag(b_s, r, kk, lane);
  };

  // One K tile: issue the DMA of tile kt+1 into `nxt`, then tile kt's MFMAs from `cur`
  // (k steps kk = 0, 1 in order, as the m16 family).  The stages are separate __shared__
  // objects named at compile time (unrolled by two), so the fragment reads of one stage are
  // not ordered behind the DMA in flight into the other.
  auto compute = [&](const char* cur) {
    const char* a_s = cur + aimg * B16_IMG;
    const char* b_s = cur + NA * B16_IMG;
    if constexpr (IM == 2) {
      b16x8_t fa[2][IM], fb[2][2];
#pragma unroll
      for (int i = 0; i < IM; ++i) fa[0][i] = fragA(a_s, i, 0);
      fb[0][0] = fragB(b_s, 0, 0);
      fb[0][1] = fragB(b_s, 1, 0);
#pragma unroll
      for (int i = 0; i < IM; ++i) fa[1][i] = fragA(a_s, i, 1);
      fb[1][0] = fragB(b_s, 0, 1);
      fb[1][1] = fragB(b_s, 1, 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int im = 0; im < IM; ++im)
#pragma unroll
          for (int in = 0; in < 2; ++in)
            acc[im][in] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[kk][im], fb[kk][in], acc[im][in], 0, 0, 0);
    } else {
      // 256-row tile: one k step's fragments at a time (the two-step form of the 128-row tile
      // left the compiler a private array here: 576 B of scratch, ~20x slower, round 6)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const b16x8_t b0 = fragB(b_s, 0, kk), b1 = fragB(b_s, 1, kk);
#pragma unroll
        for (int im = 0; im < IM; ++im) {
          const b16x8_t a = fragA(a_s, im, kk);
          acc[im][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b0, acc[im][0], 0, 0, 0);
          acc[im][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b1, acc[im][1], 0, 0, 0);
        }
      }
    }
  };
  // a stage holds K tiles kt .. kt + KT2 - 1 (those below kt_end; the condition is wave-uniform)
  auto issue_stage = [&](int kt, char* st) {
    issue(kt, st);
    if (KT2 == 2 && kt + 1 < kt_end) issue(kt + 1, st + TILE);
  };
  auto tile = [&](int kt, const char* cur, char* nxt) {
    if (kt + KT2 < kt_end) issue_stage(kt + KT2, nxt);
    compute(cur);
    if (KT2 == 2 && kt + 1 < kt_end) compute(cur + TILE);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of the next stage has landed
    __syncthreads();                                   // ... every wave's, and `cur` is no longer read
  };

  if (kt_begin < kt_end) issue_stage(kt_begin, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = kt_begin; kt < kt_end; kt += 2 * KT2) {
    tile(kt, smem, smem1);
    if (kt + KT2 >= kt_end) break;
    tile(kt + KT2, smem1, smem);
  }

#define EP_IM IM
#define EP_WTM WTM
#include "gemm_epilogue.inc"
}

// variants (gemm_f32.hip, mode GEMM_B16): 0 = 128-row tile (3 waves/SIMD), 1 = 256-row tile,
// 2 = 128-row tile with two K tiles per stage (2 waves/SIMD); all the same k order.  (Tried in
// round 6 and dropped: a 4/6-stage DMA ring and register staging (buffer_load_dwordx4 +
// ds_write_b128, 1 or 2 K tiles ahead) -- neither moved the small-grid shapes, which run at
// ~32 GB/s of operand fetch per workgroup however the fetch is issued:
// profiles/round6/b16_variants_*.txt)
template <int AL, int BL>
static void (*pick_b16(int v))(GemmParams) {
  switch (v) {
    case 0: return gemm_b16_kernel<AL, BL, 128, 3>;
    case 1: return gemm_b16_kernel<AL, BL, 256, 2>;
    case 2: return gemm_b16_kernel<AL, BL, 128, 2, 2>;
    default: return nullptr;
  }
}

}  // namespace mdemi
