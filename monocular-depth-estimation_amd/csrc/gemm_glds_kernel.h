// fp32 MFMA GEMM with direct-to-LDS operand staging (gfx950 `buffer_load_dwordx4 ... lds`):
// the pipelining variants 8..11 of the fp32 family (gemm_f32_kernel.h pick_variant) for
// dense operands (k-contiguous or m/n-contiguous, 16-B vectorisable, no load-time op).
//
// Why: the register-staged kernel spends its issue slots and VGPRs on the global loads, the
// LDS stores and the barrier around them; with every load landing in LDS by DMA a wave issues
// one buffer load per KiB of tile and nothing else (profiles/round3/gemm_study_ceilings.txt:
// without global loads the same tiles ran 118-132 TF/s against 97-114 shipped).
//
// Staging.  One wave instruction moves 64 lanes x 16 B into 1 KiB of LDS at a wave-uniform
// base (M0) + 16 * lane, so the images are lane-linear and any swizzle is applied to the
// per-lane GLOBAL address (cdna_hip_programming.md §5, "Async global->LDS copy"):
//   k-contiguous source  -> [row][k] image, BK floats per row, 16-B chunks permuted by
//     chunk ^ swz(row) (BK 32: (row >> 1) & 7; BK 16: (row >> 2) & 3) so the fragment
//     reads (ds_read_b128, 4 k of one row per lane) are bank-conflict free;
//   m/n-contiguous source -> [k][col] image, 128 columns (512 B) per k row, read with
//     ds_read_b32 (32 consecutive columns per half-wave: conflict free).
// Out-of-range rows / k chunks get the buffer offset BUF_OOB, which the descriptor's range
// check turns into zeros written to LDS: no predicates in the K loop.
//
// Pipeline: NBUF = 2 LDS stages; the DMA of K tile kt+1 is issued before tile kt's MFMAs
// and retired by `s_waitcnt vmcnt(0)` + one barrier after them (the only barrier per tile).
// Fragments of k-group g+1 are read from LDS while group g's MFMAs issue.
//
// Numerics: the MFMA k order is the family's (k-step s of group g: lane half h takes
// k = 8g + 4h + s), K is split at the same 32-element chunks, the bias-gradient row sums
// are accumulated in the register kernel's order (thread t: column quad t & 31, k rows
// t >> 5 + 8q, then the 8 partials in order) -- so these variants agree with 0..7 bit for
// bit and the per-shape autotune never changes a result.
#pragma once
#include <type_traits>

#include "common.h"
#include "gemm_core.h"

namespace mdemi {

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, const void* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds, 16, voff, 0, 0, 0);
}

template <int BK>
struct GSwz {  // chunk permutation of a [row][k] image
  static constexpr int CH = BK / 4;  // 16-B chunks per row
  __device__ static int of(int row) { return BK == 32 ? (row >> 1) & 7 : (row >> 2) & 3; }
};

// k-contiguous operand, one ROWS-row (128, or 192 for the B operand of the 192-column tile)
// [row][BK] image.  Wave w issues instructions q = w * NI + i (i < NI), each covering rows
// RPI*q .. RPI*q + RPI-1.
template <int BK, int ROWS = 128>
struct GLoadKC {
  static constexpr int CH = BK / 4, RPI = 64 / CH, NI = ROWS / RPI / 4;
  const float* base; int K;
  int voff[NI];  // byte offset of this lane's (row, chunk) within the tile, k0 = 0 (BUF_OOB: row out of range)
  int kch[NI];   // this lane's k chunk (the global chunk stored at its LDS slot)
  __device__ void init(const float* p, int64_t ld, int rows, int K_, int r0, int wid, int lane) {
    base = p + (int64_t)r0 * ld; K = K_;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = wid * NI + i, row = RPI * q + lane / CH;
      const int ch = (lane % CH) ^ GSwz<BK>::of(row);
      kch[i] = ch;
      voff[i] = r0 + row < rows ? (int)(((int64_t)row * ld + 4 * ch) * 4) : BUF_OOB;
    }
  }
  __device__ void issue(int k0, float* img, int wid) const {
    const auto rs = make_rsrc(base + k0);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = wid * NI + i;
      glds16(rs, img + q * 256, k0 + 4 * kch[i] < K ? voff[i] : BUF_OOB);
    }
  }
  // 4 consecutive k (8g + 4h .. +3) of image row r
  __device__ static float4 frag(const float* img, int r, int g, int h) {
    return *reinterpret_cast<const float4*>(img + r * BK + 4 * ((2 * g + h) ^ GSwz<BK>::of(r)));
  }
};

// m/n-contiguous operand, one [BK][128] image.  Instruction q covers k rows 2q, 2q+1.
template <int BK>
struct GLoadMN {
  static constexpr int NI = BK / 2 / 4;
  const float* base; int64_t ld; int K;
  int voff, kl;  // this lane's byte offset at k0 = 0 of instruction 0 (BUF_OOB: columns out of range), k row
  __device__ void init(const float* p, int64_t ld_, int cols, int K_, int c0, int wid, int lane) {
    base = p + c0; ld = ld_; K = K_;
    const int col = 4 * (lane & 31);
    kl = 2 * (wid * NI) + (lane >> 5);
    voff = c0 + col < cols ? (int)(((int64_t)kl * ld + col) * 4) : BUF_OOB;
  }
  __device__ void issue(int k0, float* img, int wid) const {
    const auto rs = make_rsrc(base + (int64_t)k0 * ld);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = wid * NI + i;
      const bool kin = k0 + kl + 2 * i < K;
      glds16(rs, img + q * 256, kin && voff != BUF_OOB ? voff + (int)(2 * i * ld * 4) : BUF_OOB);
    }
  }
  __device__ static float4 frag(const float* img, int r, int g, int h) {
    const float* p = img + (8 * g + 4 * h) * 128 + r;
    return make_float4(p[0], p[128], p[256], p[384]);
  }
};

// m/n-contiguous operand, columns 128 .. 191 of the 192-column tile: one [BK][64] image.
// Instruction q covers k rows 4q .. 4q+3 (lane j -> k row 4q + j/16, columns 4 (j%16) ..).
template <int BK>
struct GLoadMN64 {
  static constexpr int NI = BK / 4 / 4;
  const float* base; int64_t ld; int K;
  int voff, kl;
  __device__ void init(const float* p, int64_t ld_, int cols, int K_, int c0, int wid, int lane) {
    base = p + c0; ld = ld_; K = K_;
    const int col = 4 * (lane & 15);
    kl = 4 * (wid * NI) + (lane >> 4);
    voff = c0 + col < cols ? (int)(((int64_t)kl * ld + col) * 4) : BUF_OOB;
  }
  __device__ void issue(int k0, float* img, int wid) const {
    const auto rs = make_rsrc(base + (int64_t)k0 * ld);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = wid * NI + i;
      const bool kin = k0 + kl + 4 * i < K;
      glds16(rs, img + q * 256, kin && voff != BUF_OOB ? voff + (int)(4 * i * ld * 4) : BUF_OOB);
    }
  }
};

// 4 consecutive k (8g + 4h ..) of column c of a [BK][pitch] image (pitch 128 or 64)
__device__ __forceinline__ float4 mn_frag_pitch(const float* img, int pitch, int c, int g, int h) {
  const float* p = img + (8 * g + 4 * h) * pitch + c;
  return make_float4(p[0], p[pitch], p[2 * pitch], p[3 * pitch]);
}

template <int L, int BK, int ROWS = 128>
using GLoad = typename std::conditional<L == MDEMI_L_KCONTIG, GLoadKC<BK, ROWS>, GLoadMN<BK>>::type;

// BMT: block-tile rows (128: 2x2 waves of 64x64; 256: 2x2 waves of 128x64, A as two
// 128-row images).  BNT: block-tile columns, 128, or 192 (2x2 waves of 64x96: the N = 192 /
// 576 GEMMs of the Swin stage 0, which a 128-column tile covers in 1.5 / 4.5 tiles; B as one
// 192-row k-contiguous image, or a 128- and a 64-column m/n-contiguous image).  BK: 16 or
// 32.  OCC: waves per SIMD the register budget targets.
template <int AL, int BL, int BMT, int BK, int OCC, int BNT = 128>
__global__ __launch_bounds__(GTHREADS) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void gemm_glds_kernel(
    GemmParams p) {
  static_assert(AL != MDEMI_L_CONV && BL != MDEMI_L_CONV, "dense operands only");
  static_assert(BK == 16 || BK == 32, "BK");
  static_assert(BNT == 128 || (BNT == 192 && BMT == 128), "192-column tiles: 128 rows");
  constexpr int NA = BMT / 128, IM = BMT / 64, WTM = BMT / 2;
  constexpr int WTN = BNT / 2, IN = WTN / 32;  // wave tile columns, 32-column accumulators
  constexpr int IMG = 128 * BK;               // floats per 128-row (or 128-column) image
  constexpr int STAGE = NA * IMG + BNT * BK;  // A images + the B image(s)
  constexpr int NG = BK / 8;                  // k groups per tile
  // stage 0 is `smem` (the epilogue's split-K hand-off flag and the row-sum reduction reuse
  // it after the loop), stage 1 `smem1`
  __shared__ __attribute__((aligned(16))) float smem[STAGE];
  __shared__ __attribute__((aligned(16))) float smem1[STAGE];

  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const GemmJob job = job_of(p);
  const int b = job.b, sidx = job.sidx, tm = job.tm, tn = job.tn;
  const int bm = tm * BMT, bn = tn * BNT;

  using LA = GLoad<AL, BK>;
  using LB = GLoad<BL, BK, BNT>;
  constexpr bool B64 = BNT == 192 && BL == MDEMI_L_MNCONTIG;  // the extra 64-column B image
  LA la[NA];
  LB lb;
  GLoadMN64<BK> lb64;
#pragma unroll
  for (int a = 0; a < NA; ++a)
    la[a].init(p.A + boff(p, b, p.a_bs, p.a_bs2), p.lda, p.M, p.K, bm + 128 * a, wid, lane);
  lb.init(p.B + boff(p, b, p.b_bs, p.b_bs2), p.ldb, p.N, p.K, bn, wid, lane);
  if constexpr (B64) lb64.init(p.B + boff(p, b, p.b_bs, p.b_bs2), p.ldb, p.N, p.K, bn + 128, wid, lane);

  const int ktiles_total = (p.K + BK - 1) / BK;
  const int kt_begin = job.split ? sidx * p.ktile_per_split : 0;
  const int kt_end = job.split ? min(ktiles_total, kt_begin + p.ktile_per_split) : ktiles_total;

  floatx16 acc[IM][IN];
#pragma unroll
  for (int a = 0; a < IM; ++a)
#pragma unroll
    for (int c = 0; c < IN; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  auto issue = [&](int kt, float* st) {
#pragma unroll
    for (int a = 0; a < NA; ++a) la[a].issue(kt * BK, st + a * IMG, wid);
    lb.issue(kt * BK, st + NA * IMG, wid);
    if constexpr (B64) lb64.issue(kt * BK, st + NA * IMG + IMG, wid);
  };

  // bias-gradient row sums of an m-contiguous A, in the register kernel's order
  constexpr bool CAN_RSUM = AL == MDEMI_L_MNCONTIG;
  const bool do_rsum = CAN_RSUM && p.rowsum != nullptr && tn == 0;
  float4 rsum[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) rsum[a] = make_float4(0.f, 0.f, 0.f, 0.f);

  const int l31 = lane & 31, h = lane >> 5;
  int rA[IM];
#pragma unroll
  for (int i = 0; i < IM; ++i) rA[i] = (wm * WTM + 32 * i + l31) & 127;
  const int aimg = (wm * WTM) >> 7;
  // B fragment j: columns cb_j = wn * WTN + 32 j (+ l31); for the 192-column m/n-contiguous
  // tile, those >= 128 come from the 64-column image (a wave-uniform choice)
  auto fragB = [&](const float* b_s, int j, int g) -> float4 {
    const int cb = wn * WTN + 32 * j;
    if constexpr (B64) {
      if (cb >= 128) return mn_frag_pitch(b_s + IMG, 64, cb - 128 + l31, g, h);
      return mn_frag_pitch(b_s, 128, cb + l31, g, h);
    } else {
      return LB::frag(b_s, cb + l31, g, h);
    }
  };

  // One K tile: issue the DMA of tile kt+1 into `nxt`, then the row sums and MFMAs of tile
  // kt from `cur`.  The two stages are separate __shared__ objects and every call below
  // names them at compile time (the loop is unrolled by two), so the compiler's LDS alias
  // scopes tell it a fragment read of one stage cannot depend on the DMA in flight into the
  // other: without that it waits vmcnt(0) before the first ds_read of every tile and the
  // load no longer overlaps the MFMAs.
  auto tile = [&](int kt, const float* cur, float* nxt) {
    if (kt + 1 < kt_end) issue(kt + 1, nxt);
    if (CAN_RSUM && do_rsum) {
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int q = 0; q < BK / 8; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(cur + a * IMG + ((t >> 5) + 8 * q) * 128 + 4 * (t & 31));
          rsum[a].x += v.x; rsum[a].y += v.y; rsum[a].z += v.z; rsum[a].w += v.w;
        }
    }
    const float* a_s = cur + aimg * IMG;
    const float* b_s = cur + NA * IMG;
    float4 fa[2][IM], fb[2][IN];
#pragma unroll
    for (int i = 0; i < IM; ++i) fa[0][i] = LA::frag(a_s, rA[i], 0, h);
#pragma unroll
    for (int j = 0; j < IN; ++j) fb[0][j] = fragB(b_s, j, 0);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int c = g & 1, n = c ^ 1;
      if (g + 1 < NG) {
#pragma unroll
        for (int i = 0; i < IM; ++i) fa[n][i] = LA::frag(a_s, rA[i], g + 1, h);
#pragma unroll
        for (int j = 0; j < IN; ++j) fb[n][j] = fragB(b_s, j, g + 1);
      }
      // keep the reads of group g+1 ahead of group g's MFMAs (the scheduler would otherwise
      // sink them behind the MFMAs and expose their latency at the next group)
      __builtin_amdgcn_sched_barrier(0);
#define MDEMI_GSTEP(X)                                                                             \
  _Pragma("unroll") for (int i = 0; i < IM; ++i)                                                   \
  _Pragma("unroll") for (int j = 0; j < IN; ++j)                                                   \
    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[c][i].X, fb[c][j].X, acc[i][j], 0, 0, 0);
      MDEMI_GSTEP(x) MDEMI_GSTEP(y) MDEMI_GSTEP(z) MDEMI_GSTEP(w)
#undef MDEMI_GSTEP
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile kt+1 has landed
    __syncthreads();                                   // ... every wave's, and `cur` is no longer read
  };

  if (kt_begin < kt_end) issue(kt_begin, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = kt_begin; kt < kt_end; kt += 2) {
    tile(kt, smem, smem1);
    if (kt + 1 >= kt_end) break;
    tile(kt + 1, smem1, smem);
  }
  if (CAN_RSUM && do_rsum) {  // the 8 k-row groups (t >> 5) of each A image, in order
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
#define EP_IN IN
#define EP_WTM WTM
#define EP_WTN WTN
#include "gemm_epilogue.inc"
}

// variants 8..12 (gemm_f32.hip pick_kernel), instantiated per layout pair in gemm_glds_inst*.hip
template <int AL, int BL>
static void (*pick_glds(int v))(GemmParams) {
  if constexpr (AL == MDEMI_L_CONV || BL == MDEMI_L_CONV) {
    return nullptr;
  } else {
    switch (v) {
      case 8: return gemm_glds_kernel<AL, BL, 128, 32, 2>;
      case 9: return gemm_glds_kernel<AL, BL, 256, 16, 2>;
      case 10: return gemm_glds_kernel<AL, BL, 256, 32, 1>;
      case 11: return gemm_glds_kernel<AL, BL, 128, 16, 3>;
      case 12: return gemm_glds_kernel<AL, BL, 128, 32, 2, 192>;
      default: return nullptr;
    }
  }
}

}  // namespace mdemi
