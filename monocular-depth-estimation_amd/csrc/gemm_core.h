// Shared pieces of the GEMM kernel families (gemm_f32.hip: exact-fp32 MFMA;
// gemm_mfma16.hip: 16-bit-operand MFMA for the bf16 and split-fp32 modes):
// parameters, branch-free buffer loads, the operand loaders (dense
// k-contiguous, dense m/n-contiguous, implicit-im2col NHWC), the fused
// epilogue value and the XCD-aware tile raster.
#pragma once
#include <utility>

#include "common.h"

namespace mdemi {

// f(std::integral_constant<int, i>) for i = 0 .. N-1, expanded at compile time: the epilogue
// indexes the accumulator array with these constants, so it never depends on the unroller
// (whose give-up on the 256-row tiles' epilogue left acc[4][2] as a private array in scratch)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int GBM = 128, GBN = 128, GTHREADS = 256;
constexpr int PMN = GBM + 4;   // [k][row] image pitch (floats)
template <int BK> struct PitchK { static constexpr int v = BK + 4; };  // [row][k] image pitch

struct FastDiv {
  uint32_t mul, shift;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t c = 0;
  while ((1u << c) < d) ++c;
  const uint32_t L = 31 + c;
  return FastDiv{(uint32_t)(((uint64_t)1 << L) / d + 1), L};
}

struct GemmParams {
  int M, N, K, batch, split, ktile_per_split;
  const float* A; int64_t lda, a_bs;
  const float* B; int64_t ldb, b_bs;
  float* C; int64_t ldc, c_bs;
  float alpha, beta;
  const float* bias; int bias_mode, act;
  const float* aux; int64_t ldaux, aux_bs;
  const float* res; int64_t ldres, res_bs;
  float* pre; int64_t ldpre, pre_bs;  // optional pre-activation output
  float* rowsum;   // optional sum_k A(i,k) (A m-contiguous, batch 1): [split][M] partials or [M]
  float* slab;  // split-K partials [split][batch][M][N]
  mdemi_conv_geom cv;
  FastDiv fd_c, fd_kw, fd_ow, fd_oh;  // conv index decomposition
  int a_vec, b_vec;  // 1: 16-byte vector loads legal for this operand
  int tiles_m, tiles_n, group_m;
  int binner;  // > 1: two-level batch (mdemi_gemm_desc.batch_inner)
  int64_t a_bs2, b_bs2, c_bs2;
  const float* rowscale; FastDiv fd_rs;  // optional per-row-group scale before the residual add
  // Tail split (batch 1): row tiles [0, tiles_m1) take the whole K; the tiles_m row tiles
  // below m_split = tiles_m1 * BMT are split `split` ways (the last, partial round of
  // tiles), as is every tile of an ordinary split-K GEMM (tiles_m1 = 0).
  int tiles_m1, m_split;
  int* tile_cnt;  // non-null: the last-arriving split of a tile combines the slabs (no reduce launch)
  float* rowsum_out;  // with tile_cnt and split row-sum partials: the last arriver writes the sums here
  void* c16;  // optional bf16 copy (RNE) of the final output, C's layout: the bf16 operand of a later GEMM
};

// One thread's 4 bias-gradient row sums (rows i..i+3) of a K piece: plain stores, or
// write-through (sc1) stores when the pieces are split (the tile's last arriver may read
// them in this launch, gemm_epilogue.inc).
__device__ __forceinline__ void store_rowsum4(const GemmParams& p, int sidx, int i, float4 s4) {
  float* dst = p.rowsum + (p.split > 1 ? (int64_t)sidx * p.M : 0);
  const float v[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (i + e >= p.M) break;
    if (p.split > 1) __hip_atomic_store(dst + i + e, v[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else dst[i + e] = v[e];
  }
}

// element offset of batch entry b of an operand with outer stride s, inner stride s2
__device__ __forceinline__ int64_t boff(const GemmParams& p, int b, int64_t s, int64_t s2) {
  if (p.binner <= 1) return (int64_t)b * s;
  const int o = b / p.binner;
  return (int64_t)o * s + (int64_t)(b - o * p.binner) * s2;
}

// ---------------------------------------------------------------------------
// Branch-free operand fetch.  Dense operands use buffer loads through a
// wave-uniform descriptor rebased to the current K tile (SALU work only);
// out-of-range elements get the offset BUF_OOB, which the hardware range check
// turns into zeros.  NHWC gathers use 64-bit loads from a clamped address and
// zero the result with a select.  No per-element control flow in the K loop.
// ---------------------------------------------------------------------------
constexpr int BUF_OOB = (int)0x80000000u;
constexpr int BUF_RECORDS = 0x7fffffff;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, BUF_RECORDS, 0x00020000);
}
__device__ __forceinline__ float4 buf_ld4(__amdgpu_buffer_rsrc_t r, int off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return *reinterpret_cast<float4*>(&v);
}
__device__ __forceinline__ float buf_ld1(__amdgpu_buffer_rsrc_t r, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
// sc1 load (bypasses this CU's L1): reads bytes another workgroup stored sc1 in this launch
__device__ __forceinline__ float buf_ld1_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16));
}

// n / d for 0 <= n < 2^31 by multiply-shift (host-computed magic, exact).
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)(((uint64_t)(uint32_t)n * f.mul) >> f.shift);
}

template <int OP>
__device__ __forceinline__ float4 apply_op(float4 v) {
  if (OP == MDEMI_OP_GELU) { v.x = gelu_f(v.x); v.y = gelu_f(v.y); v.z = gelu_f(v.z); v.w = gelu_f(v.w); }
  return v;
}

// staged-image kinds
constexpr int IMG_RK = 0;  // [row][k], pitch PK
constexpr int IMG_KR = 1;  // [k][row], pitch PMN (written as float4 rows)
constexpr int IMG_KT = 2;  // [k][row], pitch GBM+2, written transposed (4x ds_write_b32) from a row-major source

template <int IMG, int BK>
struct Img {
  static constexpr int PK = PitchK<BK>::v;
  static constexpr int PT = (IMG == IMG_KT) ? GBM + 2 : PMN;
  static constexpr int floats = (IMG == IMG_RK) ? GBM * PK : BK * PT;
  // 4 consecutive MFMA k-steps (group t) for fragment row `r` of this lane half h
  __device__ static float4 frag(const float* s, int r, int t, int h) {
    if (IMG == IMG_RK) return *reinterpret_cast<const float4*>(s + r * PK + 8 * t + 4 * h);
    const float* p = s + (8 * t + 4 * h) * PT + r;
    return make_float4(p[0], p[PT], p[2 * PT], p[3 * PT]);
  }
};

// ---------------------------------------------------------------------------
// Operand loaders: each thread stages NQ = BK/8 float4 per operand per K tile.
//   row-major tile  (128 rows x BK k): f = t + 256 q -> row f/(BK/4), k-quad f%(BK/4)
//   k-major tile    (BK k x 128 cols): f = t + 256 q -> k f>>5, col-quad f&31
// ---------------------------------------------------------------------------
template <int BK>
__device__ __forceinline__ void store_rk(float* lds, int t, const float4 (&r)[BK / 8]) {
  constexpr int KQ = BK / 4, RS = 256 / KQ;
#pragma unroll
  for (int q = 0; q < BK / 8; ++q)
    *reinterpret_cast<float4*>(lds + (t / KQ + RS * q) * PitchK<BK>::v + 4 * (t % KQ)) = r[q];
}
// row-major source tile transposed into a [k][row] image (pitch 130: the 4
// k-rows a 32-lane group writes land on distinct banks)
template <int BK>
__device__ __forceinline__ void store_kt(float* lds, int t, const float4 (&r)[BK / 8]) {
  constexpr int KQ = BK / 4, RS = 256 / KQ, P = GBM + 2;
#pragma unroll
  for (int q = 0; q < BK / 8; ++q) {
    const int row = t / KQ + RS * q, k = 4 * (t % KQ);
    lds[(k + 0) * P + row] = r[q].x;
    lds[(k + 1) * P + row] = r[q].y;
    lds[(k + 2) * P + row] = r[q].z;
    lds[(k + 3) * P + row] = r[q].w;
  }
}
template <int BK>
__device__ __forceinline__ void store_kr(float* lds, int t, const float4 (&r)[BK / 8]) {
#pragma unroll
  for (int q = 0; q < BK / 8; ++q)
    *reinterpret_cast<float4*>(lds + ((t >> 5) + 8 * q) * PMN + 4 * (t & 31)) = r[q];
}

// KC selects the k mapping of the m/n-contiguous loaders: false = k rows t/32 + 8q
// (the fp32 kernel's [k][row] images), true = NQ consecutive k rows NQ*(t/32) + q per
// thread (a thread then holds a 4-col x NQ-k block it can transpose in registers).
template <int LAYOUT, int OP, bool IS_A, int BK, bool TR, bool KC = false>
struct Loader;

// dense [row][k]: thread t covers rows t/KQ + RS*q, k-quad t%KQ
template <int OP, bool IS_A, int BK, bool TR, bool KC>
struct Loader<MDEMI_L_KCONTIG, OP, IS_A, BK, TR, KC> {
  static constexpr int IMG = TR ? IMG_KT : IMG_RK, NQ = BK / 8, KQ = BK / 4, RS = 256 / KQ;
  const float* base; int K; bool vec;
  int voff[NQ]; int kq;
  __device__ void init(const float* p, int64_t ld, int rows, int K_, bool vec_, int r0, int t, const GemmParams&) {
    base = p + (int64_t)r0 * ld; K = K_; vec = vec_; kq = t % KQ;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int row = t / KQ + RS * q;
      voff[q] = r0 + row < rows ? (int)(((int64_t)row * ld + 4 * kq) * 4) : BUF_OOB;
    }
  }
  __device__ void load(int k0, float4 (&r)[NQ]) const {
    const auto rs = make_rsrc(base + k0);
    const int k = k0 + 4 * kq;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (vec) {
        r[q] = buf_ld4(rs, k < K ? voff[q] : BUF_OOB);
      } else {
        r[q].x = buf_ld1(rs, k + 0 < K ? voff[q] + 0 : BUF_OOB);
        r[q].y = buf_ld1(rs, k + 1 < K ? voff[q] + 4 : BUF_OOB);
        r[q].z = buf_ld1(rs, k + 2 < K ? voff[q] + 8 : BUF_OOB);
        r[q].w = buf_ld1(rs, k + 3 < K ? voff[q] + 12 : BUF_OOB);
      }
      r[q] = apply_op<OP>(r[q]);
    }
  }
  __device__ static void store(float* lds, int t, const float4 (&r)[NQ]) {
    if (TR) store_kt<BK>(lds, t, r); else store_rk<BK>(lds, t, r);
  }
};

// dense [k][row]: thread t covers k rows t/32 + 8q (KC: NQ*(t/32) + q), column quad t%32
template <int OP, bool IS_A, int BK, bool TR, bool KC>
struct Loader<MDEMI_L_MNCONTIG, OP, IS_A, BK, TR, KC> {
  static constexpr int IMG = IMG_KR, NQ = BK / 8, KS = KC ? 1 : 8;
  const float* base; int64_t ld; int K; bool vec;
  int voff; int kl; int cvalid;  // valid columns of this thread's quad (0..4)
  __device__ void init(const float* p, int64_t ld_, int cols, int K_, bool vec_, int c0, int t, const GemmParams&) {
    base = p + c0; ld = ld_; K = K_; vec = vec_;
    const int col = 4 * (t & 31);
    kl = KC ? NQ * (t >> 5) : (t >> 5);
    cvalid = max(0, min(4, cols - c0 - col));
    voff = (int)(((int64_t)kl * ld + col) * 4);
  }
  __device__ void load(int k0, float4 (&r)[NQ]) const {
    const auto rs = make_rsrc(base + (int64_t)k0 * ld);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool kin = k0 + kl + KS * q < K;
      const int off = voff + (int)(KS * q * ld * 4);
      if (vec) {
        r[q] = buf_ld4(rs, kin && cvalid > 0 ? off : BUF_OOB);
      } else {
        r[q].x = buf_ld1(rs, kin && cvalid > 0 ? off + 0 : BUF_OOB);
        r[q].y = buf_ld1(rs, kin && cvalid > 1 ? off + 4 : BUF_OOB);
        r[q].z = buf_ld1(rs, kin && cvalid > 2 ? off + 8 : BUF_OOB);
        r[q].w = buf_ld1(rs, kin && cvalid > 3 ? off + 12 : BUF_OOB);
      }
      r[q] = apply_op<OP>(r[q]);
    }
  }
  __device__ static void store(float* lds, int t, const float4 (&r)[NQ]) { store_kr<BK>(lds, t, r); }
};

__device__ __forceinline__ float4 gather4(const float* base, int64_t idx, bool ok) {
  const float4 v = *reinterpret_cast<const float4*>(base + (ok ? idx : 0));
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Implicit im2col of an NHWC activation, operand A (row = output pixel,
// k = (ky,kx,c)).  Requires C % 4 == 0 so a k-quad never straddles a tap.
template <int OP, int BK, bool TR, bool KC>
struct Loader<MDEMI_L_CONV, OP, true, BK, TR, KC> {
  static constexpr int IMG = TR ? IMG_KT : IMG_RK, NQ = BK / 8, KQ = BK / 4, RS = 256 / KQ;
  const float* base; mdemi_conv_geom g; FastDiv fc, fkw; int K; int kq;
  int n[NQ], iy0[NQ], ix0[NQ]; bool valid[NQ];
  __device__ void init(const float* p, int64_t, int rows, int K_, bool, int r0, int t, const GemmParams& P) {
    base = p; g = P.cv; fc = P.fd_c; fkw = P.fd_kw; K = K_; kq = t % KQ;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int i = r0 + t / KQ + RS * q;
      valid[q] = i < rows;
      const int ii = valid[q] ? i : 0;
      const int tmp = fdiv(ii, P.fd_ow), ox = ii - tmp * g.ow;
      const int nn = fdiv(tmp, P.fd_oh), oy = tmp - nn * g.oh;
      n[q] = nn;
      iy0[q] = oy * g.stride - g.pad;
      ix0[q] = ox * g.stride - g.pad;
    }
  }
  __device__ void load(int k0, float4 (&r)[NQ]) const {
    const int k = k0 + 4 * kq;
    const bool kin = k < K;
    const int kk = kin ? k : 0;
    const int tap = fdiv(kk, fc), c = kk - tap * g.c;
    const int ky = fdiv(tap, fkw), kx = tap - ky * g.kw;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      int iy = iy0[q] + ky, ix = ix0[q] + kx;
      bool ok = kin && valid[q];
      if (g.pad_mode == MDEMI_PAD_REPLICATE) {
        iy = min(max(iy, 0), g.h - 1); ix = min(max(ix, 0), g.w - 1);
      } else {
        ok = ok && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
      }
      r[q] = apply_op<OP>(gather4(base, (((int64_t)n[q] * g.h + iy) * g.w + ix) * g.c + c, ok));
    }
  }
  __device__ static void store(float* lds, int t, const float4 (&r)[NQ]) {
    if (TR) store_kt<BK>(lds, t, r); else store_rk<BK>(lds, t, r);
  }
};

// Implicit im2col, operand B (weight gradients): B(k, j) with k = output pixel,
// j = (ky,kx,c); staged k-major like a dense [k][col] operand.
template <int OP, int BK, bool TR, bool KC>
struct Loader<MDEMI_L_CONV, OP, false, BK, TR, KC> {
  static constexpr int IMG = IMG_KR, NQ = BK / 8, KS = KC ? 1 : 8;
  const float* base; mdemi_conv_geom g; FastDiv fow, foh; int K; int kl;
  int c, ky, kx; bool jvalid;
  __device__ void init(const float* p, int64_t, int cols, int K_, bool, int c0, int t, const GemmParams& P) {
    base = p; g = P.cv; fow = P.fd_ow; foh = P.fd_oh; K = K_; kl = KC ? NQ * (t >> 5) : (t >> 5);
    const int j = c0 + 4 * (t & 31);
    jvalid = j < cols;
    const int jj = jvalid ? j : 0;
    const int tap = fdiv(jj, P.fd_c);
    c = jj - tap * g.c;
    ky = fdiv(tap, P.fd_kw);
    kx = tap - ky * g.kw;
  }
  __device__ void load(int k0, float4 (&r)[NQ]) const {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int k = k0 + kl + KS * q;
      bool ok = jvalid && k < K;
      const int kk = ok ? k : 0;
      const int tmp = fdiv(kk, fow), ox = kk - tmp * g.ow;
      const int nn = fdiv(tmp, foh), oy = tmp - nn * g.oh;
      int iy = oy * g.stride - g.pad + ky, ix = ox * g.stride - g.pad + kx;
      if (g.pad_mode == MDEMI_PAD_REPLICATE) {
        iy = min(max(iy, 0), g.h - 1); ix = min(max(ix, 0), g.w - 1);
      } else {
        ok = ok && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
      }
      r[q] = apply_op<OP>(gather4(base, (((int64_t)nn * g.h + iy) * g.w + ix) * g.c + c, ok));
    }
  }
  __device__ static void store(float* lds, int t, const float4 (&r)[NQ]) { store_kr<BK>(lds, t, r); }
};


__device__ __forceinline__ float epilogue_value(const GemmParams& p, int b, int i, int j, float acc) {
  float v = p.alpha * acc;
  if (p.beta != 0.f) v += p.beta * p.C[boff(p, b, p.c_bs, p.c_bs2) + (int64_t)i * p.ldc + j];
  if (p.bias_mode == MDEMI_BIAS_COL) v += p.bias[j];
  else if (p.bias_mode == MDEMI_BIAS_ROW) v += p.bias[i];
  if (p.pre) p.pre[(int64_t)b * p.pre_bs + (int64_t)i * p.ldpre + j] = v;
  if (is_grad_act(p.act)) v *= aux_grad(p.act, p.aux[(int64_t)b * p.aux_bs + (int64_t)i * p.ldaux + j]);
  else if (p.act != MDEMI_ACT_NONE) v = apply_act(p.act, v);
  if (p.rowscale) v *= p.rowscale[fdiv(i, p.fd_rs)];
  if (p.res) v += p.res[(int64_t)b * p.res_bs + (int64_t)i * p.ldres + j];
  return v;
}

// tile (tm, tn) for a linear workgroup id over tiles_m x tiles_n tiles: XCD-aware
// remap (blocks b, b+8, ... share an XCD), then grouped raster so concurrently running
// tiles of one XCD reuse A row-panels (group_m rows of tiles) and B column-panels.
// XCD-aware linear order: workgroup ids b, b+8, ... (one XCD) take one contiguous range
// of [0, n), so neighbouring jobs share that XCD's L2.
__device__ __forceinline__ int xcd_lin(int bid, int n) {
  const int q = n / 8, r = n % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ void tile_of(const GemmParams& p, int bid, int ntiles, int tiles_m, int& tm, int& tn,
                                        bool remap = true) {
  if (p.group_m <= 0) {  // plain raster: n fastest
    tm = bid / p.tiles_n;
    tn = bid % p.tiles_n;
    return;
  }
  const int lin = remap ? xcd_lin(bid, ntiles) : bid;
  const int per_group = p.group_m * p.tiles_n;
  const int grp = lin / per_group;
  const int first_m = grp * p.group_m;
  const int gm = min(tiles_m - first_m, p.group_m);
  const int in_grp = lin % per_group;
  tm = first_m + in_grp % gm;
  tn = in_grp / gm;
}

// What one workgroup computes: the whole-K tiles of the leading region come first in
// launch order, then the split region's pieces (all tiles' piece 0, then piece 1, ...).
struct GemmJob {
  int b, sidx, tm, tn, cid;  // cid: counter slot of a split tile
  bool split;
};
__device__ __forceinline__ GemmJob job_of(const GemmParams& p) {
  GemmJob j;
  const int n1 = p.tiles_m1 * p.tiles_n;
  int bid = blockIdx.x;
  if (bid < n1) {
    j.b = 0; j.sidx = 0; j.split = false; j.cid = 0;
    tile_of(p, bid, n1, p.tiles_m1, j.tm, j.tn);
    return j;
  }
  bid -= n1;
  const int n2 = p.tiles_m * p.tiles_n;
  // The XCD remap runs over all (batch entry, K piece, tile) jobs, piece-major: every tile
  // of one K piece (and of one batch entry) lands on one XCD, so a piece's operand rows --
  // e.g. the NHWC pixels the im2col columns of a weight-gradient GEMM gather once per
  // tap -- are fetched into one L2 instead of up to eight.
  if (p.group_m > 0) bid = xcd_lin(bid, n2 * p.batch * p.split);
  const int zb = bid / n2, t2 = bid - zb * n2;
  j.b = zb / p.split;
  j.sidx = zb - j.b * p.split;
  j.split = p.split > 1;
  int tm2;
  tile_of(p, t2, n2, p.tiles_m, tm2, j.tn, false);
  j.tm = p.tiles_m1 + tm2;
  j.cid = j.b * n2 + tm2 * p.tiles_n + j.tn;
  return j;
}

// precision modes of the GEMM entry points
constexpr int GEMM_F32 = 0;   // exact-product fp32 MFMA (gemm_f32.hip)
constexpr int GEMM_BF16 = 1;  // bf16 operands, fp32 accumulate (gemm_mfma16.hip, NP = 1)
constexpr int GEMM_F32E = 2;  // fp32 as three bf16 planes, six products (gemm_mfma16.hip, NP = 3)
constexpr int GEMM_B16 = 3;   // bf16 operands in HBM, direct-to-LDS (gemm_b16_kernel.h); numerics of GEMM_BF16

void (*pick_kernel_m16(int al, int bl, int aop, int bop, int np, int v))(GemmParams);
void (*pick_kernel_b16(int al, int bl, int v))(GemmParams);

}  // namespace mdemi
