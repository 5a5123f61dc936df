// Fused (shifted-)window multi-head attention with relative position bias.
//
// Reference semantics (one (window, head) per workgroup):
//   SwinTransformerBlock.forward  swin_transformer.py:201-240  (pad, roll,
//       window_partition, window_reverse, roll back, crop)
//   WindowAttention.forward       swin_transformer.py:119-141  (q*scale, QK^T,
//       + relative_position_bias_table[relative_position_index], + mask,
//       softmax, PV)
//   BasicLayer.forward mask       swin_transformer.py:361-380  (-100 between
//       different shift regions)
//   CRF variant                   newcrf_layers.py:110-149, 207-251 (q,k from
//       the qk Linear, v from the padded/rolled coarse prediction)
// Pad/roll/partition are index maps on the token-major [B,H,W] rows: a window
// token (ty,tx) of window (b,wy,wx) sits at rolled-padded (py,px) =
// (wy*WS+ty, wx*WS+tx) and reads original padded (oy,ox) = ((py+s)%Hp,
// (px+s)%Wp); it is a pad token when oy>=H or ox>=W.  The mask region of a
// rolled-padded coordinate is 0 / 1 / 2 for [0,Hp-WS) / [Hp-WS,Hp-s) / [Hp-s,Hp).
//
// Work per (window, head) is 2*N*N*HD FMAs with N = 49: small (fp32 MFMA has
// the same FLOP rate as the f32 VALU and 49 pads to 64), so the kernels are
// VALU + LDS-broadcast (lane = token, the other side's rows broadcast from
// LDS); the forward keeps the score row in registers (N compile-time) and
// saves each row's log-sum-exp for the backward.
#include "common.h"

namespace mdemi {

struct WinGeom {
  int B, H, W, Hp, Wp, nWh, nWw, shift, heads;
};

template <int WS>
struct Win {
  int b, wy, wx;
  __device__ Win(const WinGeom& g, int win) {
    wx = win % g.nWw;
    const int t = win / g.nWw;
    wy = t % g.nWh;
    b = t / g.nWh;
  }
  // row of window token t in the unpadded token-major tensor, -1 for pad
  __device__ int row(const WinGeom& g, int t) const {
    const int py = wy * WS + t / WS, px = wx * WS + t % WS;
    int oy = py + g.shift, ox = px + g.shift;
    if (oy >= g.Hp) oy -= g.Hp;
    if (ox >= g.Wp) ox -= g.Wp;
    if (oy >= g.H || ox >= g.W) return -1;
    return (b * g.H + oy) * g.W + ox;
  }
  __device__ int region(const WinGeom& g, int t) const {
    const int py = wy * WS + t / WS, px = wx * WS + t % WS;
    const int rh = py < g.Hp - WS ? 0 : (py < g.Hp - g.shift ? 1 : 2);
    const int rw = px < g.Wp - WS ? 0 : (px < g.Wp - g.shift ? 1 : 2);
    return rh * 3 + rw;
  }
};

template <int WS>
__device__ __forceinline__ int rpb_index(int i, int j) {
  return (i / WS - j / WS + WS - 1) * (2 * WS - 1) + (i % WS - j % WS + WS - 1);
}

template <int HD>
__device__ __forceinline__ void load_row(float4 (&dst)[HD / 4], const float* src) {
#pragma unroll
  for (int q = 0; q < HD / 4; ++q) dst[q] = reinterpret_cast<const float4*>(src)[q];
}

__device__ __forceinline__ float4 ld_tok4(const float* base, int64_t ld, int row, const float* pad, int off) {
  if (row >= 0) return *reinterpret_cast<const float4*>(base + (int64_t)row * ld + off);
  if (pad) return *reinterpret_cast<const float4*>(pad + off);
  return make_float4(0.f, 0.f, 0.f, 0.f);
}

// all-zero source row for padding tokens (never written)
__device__ float g_wa_zero[128];

// start of the row that window token data comes from: the token's row, the
// pad vector (Linear bias) for pad tokens, or zeros (CRF v pads, MFMA padding)
__device__ __forceinline__ const float* tok_src(const float* base, int64_t ld, int row, const float* pad, bool real) {
  const float* padsrc = pad ? pad : g_wa_zero;
  return !real ? g_wa_zero : (row >= 0 ? base + (int64_t)row * ld : padsrc);
}

__device__ __forceinline__ float dot4(const float4& a, const float4& b) {
  return fmaf(a.x, b.x, fmaf(a.y, b.y, fmaf(a.z, b.z, a.w * b.w)));
}

struct WinParams {
  WinGeom g;
  float scale;
  const float* q; const float* k; int64_t qk_ld;
  const float* q_pad; const float* k_pad;
  const float* v; int64_t v_ld; const float* v_pad;
  const float* rpb;
  float* out; int64_t out_ld;
  float* lse;  // [nwin][heads][N] log-sum-exp of each score row (+inf for pad queries)
  const float* dout;
  float* dq; float* dk; int64_t dqk_ld;
  float* dv; int64_t dv_ld;
  float* partial;  // [nwin][heads][T + 2*HD]: bias-table gradient, pad-key k / v gradient sums
  int off32;       // every row * ld of the backward's column operands fits a 24x24 -> 32-bit multiply
};

// ---------------------------------------------------------------------------
// MFMA formulation.  One wave owns one (window, head) item; a workgroup runs
// WA_WAVES items.  Tokens are padded 49 -> 64 and every product is a 64x64x32
// (or 32x64x64) tile product on v_mfma_f32_32x32x2_f32.  MFMA lane maps (the
// k-step s of a 32-deep product uses, in lane half h, element
// d(s,h) = 8*(s>>2) + 4*h + (s&3), so one float4 register per 4 steps):
//   A[i][k]: lane l gives A[l&31][d(s, l>>5)]     B[k][j]: lane l gives B[d(s, l>>5)][l&31]
//   C[i][j]: lane l, reg r holds C[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]
// A score tile computed as S^T = K Q^T (rows = keys, columns = queries) leaves
// one query per lane column, so the softmax over keys is a per-lane reduction
// plus one cross-half shuffle, and the tile feeds the next product directly
// as its B operand (k-step s <-> accumulator register s, rows r = s).
// Relative-position bias and MFMA padding (-inf for keys >= 49) are
// pre-arranged per head in accumulator order (wa_bias_kernel) and loaded as
// the accumulator's initial value; the shift mask (-100 across regions) is
// added only in the last row/column of windows, the only ones it touches.
// ---------------------------------------------------------------------------
constexpr int WA_WAVES = 4, WA_NP = 64, WA_HD = 32, WA_N = 49, WA_T = 169;
typedef float wa_f16x __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float f4c(const float4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}
__device__ __forceinline__ wa_f16x mfma32(float a, float b, wa_f16x c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// accumulator register r of lane half h -> row within the 32-row tile
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// the lane's 16 operand values of window token `tok` (d = 8g + 4h + c), scaled
__device__ __forceinline__ void load_frag(float4 (&f)[4], const float* base, int64_t ld, int row, const float* pad,
                                          bool real, int col0, int h, float scale) {
  const float* src = tok_src(base, ld, row, pad, real);
  src = src == g_wa_zero ? src : src + col0;  // the zero row serves every head
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    float4 v = *reinterpret_cast<const float4*>(src + 8 * g4 + 4 * h);
    v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
    f[g4] = v;
  }
}

// init accumulators [a][b] from a per-head bias image laid out [a][b][lane][16]
__device__ __forceinline__ void load_bias(wa_f16x (&acc)[2][2], const float* img, int lane) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const float4* src = reinterpret_cast<const float4*>(img + ((a * 2 + b) * 64 + lane) * 16);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const float4 v = src[q4];
        acc[a][b][4 * q4 + 0] = v.x; acc[a][b][4 * q4 + 1] = v.y;
        acc[a][b][4 * q4 + 2] = v.z; acc[a][b][4 * q4 + 3] = v.w;
      }
    }
}

// acc[a][b] (+)= sum_s A_a(s) B_b(s) over the 32-deep head dimension
__device__ __forceinline__ void mma_hd(wa_f16x (&acc)[2][2], const float4 (&fa)[2][4], const float4 (&fb)[2][4]) {
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(f4c(fa[a][g4], c), f4c(fb[b][g4], c), acc[a][b]);
}

// out[nt] (+)= sum over 64 tokens t of Rows[t][l&31] * Acc[t-tile][nt][reg(t)], i.e. an
// [32 x 64] x [64 x 32] product whose A comes from a [64][32] LDS row image and whose
// B is a score tile; token-tile 1 steps with every token >= 56 are skipped (all padding).
__device__ __forceinline__ void mma_tok(wa_f16x (&out)[2], const float (*rows)[WA_HD], const wa_f16x (&acc)[2][2],
                                        int l31, int h) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < (t == 0 ? 16 : 12); ++s) {
      const float a = rows[t * 32 + acc_row(s, h)][l31];
#pragma unroll
      for (int n = 0; n < 2; ++n) out[n] = mfma32(a, acc[t][n][s], out[n]);
    }
}

// Ordering of a wave's own LDS traffic (every LDS image below is private to
// one wave): the wave's DS instructions execute in issue order, so a compiler
// fence + wave barrier is enough -- no workgroup barrier couples the four
// independent (window, head) items of a workgroup.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct WaItem {
  int item, win, hh;
  bool active;
};
__device__ __forceinline__ WaItem wa_item(const WinParams& p, int nitems) {
  WaItem it;
  it.item = blockIdx.x * WA_WAVES + (threadIdx.x >> 6);
  it.active = it.item < nitems;
  const int i = it.active ? it.item : 0;
  it.win = i / p.g.heads;
  it.hh = i % p.g.heads;
  return it;
}

// per-wave region ids (shift mask) and "needs mask" flag
__device__ __forceinline__ bool wa_regions(const WinParams& p, const Win<7>& w, int8_t* reg, int lane) {
  const bool border = p.g.shift > 0 && (w.wy == p.g.nWh - 1 || w.wx == p.g.nWw - 1);
  if (border) reg[lane] = lane < WA_N ? (int8_t)w.region(p.g, lane) : (int8_t)0;
  return border;
}

template <int WS, int HD>
__global__ __launch_bounds__(256) void winattn_fwd_kernel(WinParams p, const float* __restrict__ biasT, int nitems) {
  static_assert(WS == 7 && HD == WA_HD, "MFMA window attention is built for 7x7 windows, head_dim 32");
  __shared__ float Vs[WA_WAVES][WA_NP][WA_HD];
  __shared__ int8_t regs[WA_WAVES][WA_NP];
  const WinGeom& g = p.g;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, l31 = lane & 31, h = lane >> 5;
  const WaItem it = wa_item(p, nitems);
  const Win<WS> w(g, it.win);
  const int col0 = it.hh * HD;
  for (int e = lane; e < WA_NP * HD / 4; e += 64) {
    const int tok = e >> 3, c4 = e & 7;
    const float4 v = tok < WA_N ? ld_tok4(p.v, p.v_ld, w.row(g, tok), p.v_pad, col0 + 4 * c4)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(&Vs[wv][tok][4 * c4]) = v;
  }
  const bool border = wa_regions(p, w, regs[wv], lane);
  wa_f16x s[2][2];  // S^T [key tile][query tile]
  load_bias(s, biasT + (size_t)it.hh * 4096, lane);
  {
    float4 kf[2][4], qf[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int tok = t * 32 + l31;
      const bool real = tok < WA_N;
      const int row = real ? w.row(g, tok) : -1;
      load_frag(kf[t], p.k, p.qk_ld, row, p.k_pad, real, col0, h, 1.f);
      load_frag(qf[t], p.q, p.qk_ld, row, p.q_pad, real, col0, h, p.scale);
    }
    mma_hd(s, kf, qf);
  }
  wave_lds_sync();  // Vs, regs
  if (border) {
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int rq = regs[wv][n * 32 + l31];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (regs[wv][t * 32 + acc_row(r, h)] != rq) s[t][n][r] -= 100.f;
    }
  }
  float lse[2];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaxf(m, s[t][n][r]);
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __expf(s[t][n][r] - m);
        s[t][n][r] = e;
        l += e;
      }
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.f / l;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[t][n][r] *= inv;
    lse[n] = m + __logf(l);
  }
  wa_f16x o[2];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[n][r] = 0.f;
  mma_tok(o, Vs[wv], s, l31, h);  // O^T[d][q] = sum_key V[key][d] P^T[key][q]
  if (!it.active) return;
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int q = n * 32 + l31;
    if (q >= WA_N) continue;
    const int row = w.row(g, q);
    if (p.lse && h == 0) p.lse[(int64_t)it.item * WA_N + q] = row >= 0 ? lse[n] : INFINITY;
    if (row < 0) continue;  // pad query: cropped away
    float* dst = p.out + (int64_t)row * p.out_ld + col0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
      *reinterpret_cast<float4*>(dst + 8 * a + 4 * h) =
          make_float4(o[n][4 * a], o[n][4 * a + 1], o[n][4 * a + 2], o[n][4 * a + 3]);
  }
}

// Fused backward: one wave per (window, head), one pass over Q/K/V/O/dO.
// In the S^T orientation of the forward (rows = keys in registers, columns =
// queries on lanes) the wave recomputes P^T = exp(S^T - lse) and
// dP^T = V dO^T, forms dS^T = P^T (dP^T - D) with D = rowsum(dO o O), and
//   dQ^T[d][q]  = sum_key K[key][d] dS^T[key][q]     (contracts the register rows)
//   dK[key][d]  = sum_q dS^T[key][q] (scale Q)[q][d] (contracts the lane columns)
//   dV[key][d]  = sum_q P^T[key][q] dO[q][d]
// The two products that contract over queries read the score tile back from
// a per-wave [key][query] LDS image (pitch 65: conflict-free both ways), so
// no score is computed twice.  The per-lane operand columns (K[key][l31],
// Q[q][l31], dO[q][l31]) come straight from global rows (L2 hits).  The
// relative-position-bias gradient is gathered through per-wave LDS atomics;
// pad keys (whose k / v were the Linear bias) fold into per-item sums.
#ifdef WA_OCC3  // measured alternative (tools/wa_study.sh wa_occ3 -DWA_OCC3): 2.6 % slower per NYU step
// score image of 56 key rows (keys >= 56 are padding: never stored, only read as discarded
// MFMA rows) and pitch 57 (>= the 50 query columns the products read; odd: conflict-free
// column reads): 53 KB per workgroup -> 3 workgroups per CU
constexpr int WA_TR = 56, WA_TP = 57;
#else
constexpr int WA_TR = WA_NP, WA_TP = WA_NP + 1;
#endif

// Column fetch for a window token through the wave's row table (rowtab[tok] =
// the token's row, -1 for a pad token, -2 for MFMA padding): value of column
// `col` with the forward's pad / zero semantics, branch-free.
__device__ __forceinline__ float col_val(const float* base, int64_t ld, const float* pad, int row, int col) {
  const float* src = row >= 0 ? base + (int64_t)row * ld + col : ((row == -1 && pad) ? pad + col : g_wa_zero + (col & 31));
  return *src;
}

// compile-time relative-position-table column of key token `key`
__host__ __device__ constexpr int key_tab(int key) { return (key / 7) * 13 + key % 7; }

// Fast path of a window with no pad tokens (all 49 tokens are real rows, tokens >= 49 are MFMA
// padding): which window tokens ti*32 + acc_row(r, h) / 2j + h are real is known at compile
// time except for one register / pair, where it depends on the lane half.
//   kind 0: real in both halves, 1: real only in half 0, 2: padding in both
__host__ __device__ constexpr int acc_tok_kind(int ti, int r) {
  return (ti * 32 + (r & 3) + 8 * (r >> 2) + 4 >= WA_N) ? ((ti * 32 + (r & 3) + 8 * (r >> 2) >= WA_N) ? 2 : 1) : 0;
}
__host__ __device__ constexpr int pair_tok_kind(int j) { return 2 * j + 1 >= WA_N ? (2 * j >= WA_N ? 2 : 1) : 0; }

// Per-lane column values c[j] = scale * X[token 2j + h][col0 + l31] (j < 25).  FAST: every
// token < 49 is a real row (no pad tokens in the window) and row * ld fits 32 bits, so the
// address is one 24-bit multiply-add from the row table; token 49 (j = 24, half 1) is padding.
template <bool FAST>
__device__ __forceinline__ void fetch_pairs(float (&c)[25], const float* base, int64_t ld, const float* pad,
                                            const int* rt, int col0, int l31, int h, float scale) {
  if (FAST) {
    const float* cb = base + col0 + l31;
#pragma unroll
    for (int j = 0; j < 25; ++j) {
      const int kind = pair_tok_kind(j);
      const float v = cb[__umul24((unsigned)rt[kind ? 2 * j : 2 * j + h], (unsigned)ld)];
      c[j] = (kind && h) ? 0.f : scale * v;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 25; ++j) c[j] = scale * col_val(base, ld, pad, rt[2 * j + h], col0 + l31);
  }
}

// c[t][r] = X[token t*32 + acc_row(r, h)][col0 + l31], the key rows of the accumulator layout
template <bool FAST>
__device__ __forceinline__ void fetch_keys(float (&c)[2][16], const float* base, int64_t ld, const float* pad,
                                           const int* rt, int col0, int l31, int h) {
  if (FAST) {
    const float* cb = base + col0 + l31;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kind = acc_tok_kind(t, r);
        if (kind == 2) {
          c[t][r] = 0.f;
          continue;
        }
        const float v = cb[__umul24((unsigned)rt[kind ? t * 32 + acc_row(r, 0) : t * 32 + acc_row(r, h)], (unsigned)ld)];
        c[t][r] = (kind && h) ? 0.f : v;
      }
  } else {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) c[t][r] = col_val(base, ld, pad, rt[t * 32 + acc_row(r, h)], col0 + l31);
  }
}

template <int WS, int HD>
#ifdef WA_OCC3
#define WA_BWD_OCC 3
#else
#define WA_BWD_OCC 2
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WA_BWD_OCC, WA_BWD_OCC))) void winattn_bwd_kernel(
    WinParams p, const float* __restrict__ biasT, int nitems) {
  __shared__ float tbuf[WA_WAVES][WA_TR][WA_TP];
  __shared__ float padk[WA_WAVES][WA_HD], padv[WA_WAVES][WA_HD];
  __shared__ int8_t regs[WA_WAVES][WA_NP];
  __shared__ int rowtab[WA_WAVES][WA_NP];
  const WinGeom& g = p.g;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, l31 = lane & 31, h = lane >> 5;
  const WaItem it = wa_item(p, nitems);
  const Win<WS> w(g, it.win);
  const int col0 = it.hh * HD;
  // the saved log-sum-exp of this lane's two query columns, first: the softmax gradient waits on it
  float lse[2];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int q = n * 32 + l31;
    lse[n] = (q < WA_N) ? p.lse[(int64_t)it.item * WA_N + q] : INFINITY;  // +inf: P = 0
  }
  const int myrow = lane < WA_N ? w.row(g, lane) : -2;
  rowtab[wv][lane] = myrow;
  if (lane < HD) { padk[wv][lane] = 0.f; padv[wv][lane] = 0.f; }
  const bool border = wa_regions(p, w, regs[wv], lane);
  // wave-uniform: a window without pad tokens (most of them) takes the predicate-free fast path
  const bool fast = p.off32 && __ballot(myrow == -1) == 0;

  wa_f16x s[2][2], dp[2][2];  // S^T / P^T and dP^T / dS^T  [key tile][query tile]
  load_bias(s, biasT + (size_t)it.hh * 4096, lane);
  int trow[2];
  bool treal[2];
  {
    float4 kf[2][4], qf[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int tok = t * 32 + l31;
      treal[t] = tok < WA_N;
      trow[t] = treal[t] ? w.row(g, tok) : -1;
      load_frag(kf[t], p.k, p.qk_ld, trow[t], p.k_pad, treal[t], col0, h, 1.f);
      load_frag(qf[t], p.q, p.qk_ld, trow[t], p.q_pad, treal[t], col0, h, p.scale);
    }
    mma_hd(s, kf, qf);  // S^T[key][q]
  }
  wave_lds_sync();  // pads, regs, rowtab
  if (border) {  // shift mask (-100 across regions): last window row / column only
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int rq = regs[wv][n * 32 + l31];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (regs[wv][t * 32 + acc_row(r, h)] != rq) s[t][n][r] -= 100.f;
    }
  }
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[t][n][r] = __expf(s[t][n][r] - lse[n]);  // P^T
  // ---- products over the score tiles, each read back from the per-wave LDS image ----
  auto to_lds = [&](const wa_f16x (&x)[2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#ifdef WA_OCC3
          if (t * 32 + acc_row(r, 0) >= WA_TR || (n == 1 && l31 >= WA_TP - 32)) continue;
#endif
          tbuf[wv][t * 32 + acc_row(r, h)][n * 32 + l31] = x[t][n][r];
        }
  };
  // acc[ti][r] = sum_q tbuf[ti*32 + l31][q] * col[q], q = 2j + h; row key = ti*32 + acc_row(r, h), column d = l31
  auto key_side = [&](const float (&colv)[25], float* gbase, int64_t gld, float* padacc) {
    wa_f16x acc[2];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[ti][r] = 0.f;
#pragma unroll
    for (int j = 0; j < 25; ++j)
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) acc[ti] = mfma32(tbuf[wv][ti * 32 + l31][2 * j + h], colv[j], acc[ti]);
    if (!it.active) return;
    if (fast) {
      float* gb = gbase + col0 + l31;
      const int* rt = rowtab[wv];
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kind = acc_tok_kind(ti, r);
          if (kind == 2 || (kind == 1 && h)) continue;
          gb[__umul24((unsigned)rt[ti * 32 + acc_row(r, h)], (unsigned)gld)] = acc[ti][r];
        }
      return;
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rowtab[wv][ti * 32 + acc_row(r, h)];
        if (row >= 0) gbase[(int64_t)row * gld + col0 + l31] = acc[ti][r];
        else if (row == -1) atomicAdd(&padacc[l31], acc[ti][r]);  // pad key: into the Linear-bias gradient
      }
  };
  // dV[key][d] = sum_q P^T[key][q] dO[q][d]; P^T leaves the registers here and is read back
  // from LDS for dS, so P^T and dP^T are never live together
  {
    to_lds(s);
    wave_lds_sync();
    float dc[25];
    if (fast) fetch_pairs<true>(dc, p.dout, p.out_ld, nullptr, rowtab[wv], col0, l31, h, 1.f);
    else fetch_pairs<false>(dc, p.dout, p.out_ld, nullptr, rowtab[wv], col0, l31, h, 1.f);
    key_side(dc, p.dv, p.dv_ld, padv[wv]);
  }
  float D[2];
  {
    float4 vf[2][4], df[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      // dO / O exist only for real (non-pad) query rows: pad and padding queries get 0
      const bool qo = treal[t] && trow[t] >= 0;
      load_frag(vf[t], p.v, p.v_ld, trow[t], p.v_pad, treal[t], col0, h, 1.f);
      load_frag(df[t], p.dout, p.out_ld, trow[t], nullptr, qo, col0, h, 1.f);
      float4 of[4];
      load_frag(of, p.out, p.out_ld, trow[t], nullptr, qo, col0, h, 1.f);
      float part = 0.f;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) part += dot4(df[t][g4], of[g4]);
      D[t] = part + __shfl_xor(part, 32, 64);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) dp[a][b][r] = 0.f;
    mma_hd(dp, vf, df);  // dP^T[key][q] = sum_d V[key][d] dO[q][d]
  }
  // dS^T = P^T (dP^T - D), P^T read back from the LDS image (0 where the image has no slot:
  // padding keys / queries)
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float pr;
#ifdef WA_OCC3
        if (t * 32 + acc_row(r, 0) >= WA_TR) pr = 0.f;
        else if (n == 1) pr = l31 < WA_TP - 32 ? tbuf[wv][t * 32 + acc_row(r, h)][32 + min(l31, WA_TP - 33)] : 0.f;
        else
#endif
        pr = tbuf[wv][t * 32 + acc_row(r, h)][n * 32 + l31];
        dp[t][n][r] = pr * (dp[t][n][r] - D[n]);
      }
  float kc[2][16];
  if (fast) fetch_keys<true>(kc, p.k, p.qk_ld, p.k_pad, rowtab[wv], col0, l31, h);
  else fetch_keys<false>(kc, p.k, p.qk_ld, p.k_pad, rowtab[wv], col0, l31, h);
  wave_lds_sync();  // every P^T read done
  to_lds(dp);
  wave_lds_sync();
  float qc[25];
  if (fast) fetch_pairs<true>(qc, p.q, p.qk_ld, p.q_pad, rowtab[wv], col0, l31, h, p.scale);
  else fetch_pairs<false>(qc, p.q, p.qk_ld, p.q_pad, rowtab[wv], col0, l31, h, p.scale);
  // dQ^T[d][q] = sum_key K[key][d] dS^T[key][q]  (K columns from global, dS^T from LDS)
  {
    wa_f16x dq[2];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[n][r] = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < (t == 0 ? 16 : 12); ++r)  // keys >= 56: all padding
#pragma unroll
        for (int n = 0; n < 2; ++n)
          dq[n] = mfma32(kc[t][r], tbuf[wv][t * 32 + acc_row(r, h)][n * 32 + l31], dq[n]);
    if (it.active) {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if (!treal[n] || trow[n] < 0) continue;  // padding / pad query: cropped away
        float* dst = p.dq + (int64_t)trow[n] * p.dqk_ld + col0;
#pragma unroll
        for (int a = 0; a < 4; ++a)
          *reinterpret_cast<float4*>(dst + 8 * a + 4 * h) =
              make_float4(dq[n][4 * a] * p.scale, dq[n][4 * a + 1] * p.scale, dq[n][4 * a + 2] * p.scale,
                          dq[n][4 * a + 3] * p.scale);
      }
    }
  }
  // dK[key][d] = sum_q dS^T[key][q] (scale Q)[q][d]
  key_side(qc, p.dk, p.dqk_ld, padk[wv]);
  // Relative-position-bias gradient from the dS^T image still in LDS, deterministic and
  // without atomics: with key (ky, kx), query (qy, qx), table slot (qy-ky+6)*13 + (qx-kx+6).
  // Stage 1: lane (ky, qy) sums the 13 diagonals of its 7x7 block, E[ky][qy][dx] =
  //   sum_kx dS^T[(ky,kx)][(qy,kx+dx)] (compile-time LDS offsets and register indices).
  // Stage 2: slot (dy, dx) = sum_ky E[ky][ky+dy][dx], E staged through the same LDS image.
  float E[13];
#pragma unroll
  for (int e = 0; e < 13; ++e) E[e] = 0.f;
  const int sky = lane / WS, sqy = lane - sky * WS;
  if (lane < WA_N) {
    const float* blk = &tbuf[wv][sky * WS][sqy * WS];
#pragma unroll
    for (int kx = 0; kx < WS; ++kx)
#pragma unroll
      for (int qx = 0; qx < WS; ++qx) E[qx - kx + WS - 1] += blk[kx * WA_TP + qx];
  }
  wave_lds_sync();  // every read of the dS^T image done
  constexpr int ND = 2 * WS - 1;
  float* Eb = &tbuf[wv][0][0];  // [ky][qy][dx]
  if (lane < WA_N) {
#pragma unroll
    for (int e = 0; e < ND; ++e) Eb[lane * ND + e] = E[e];
  }
  wave_lds_sync();  // E, pads complete
  if (it.active) {
    float* P = p.partial + (int64_t)it.item * (WA_T + 2 * HD);
    for (int e = lane; e < WA_T; e += 64) {
      const int dy = e / ND - (WS - 1), dxi = e % ND;
      const int ky0 = max(0, -dy), ky1 = min(WS - 1, WS - 1 - dy);
      float acc = 0.f;
      for (int ky = ky0; ky <= ky1; ++ky) acc += Eb[(ky * WS + ky + dy) * ND + dxi];
      P[e] = acc;
    }
    if (lane < HD) {
      P[WA_T + lane] = padk[wv][lane];
      P[WA_T + HD + lane] = padv[wv][lane];
    }
  }
}

// Per-head bias images in accumulator order [a][b][lane][r] (a, b = 32-row /
// 32-column tiles): T (rows = keys, cols = queries) for the forward and the
// query-side backward, N (rows = queries, cols = keys) for the key side.
// value = table[rpb_index(q, key)][head]; -inf for MFMA-padding keys (>= 49),
// 0 for padding queries.
__global__ __launch_bounds__(256) void wa_bias_kernel(const float* __restrict__ rpb, int heads, float* biasT,
                                                      float* biasN) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= heads * 4096) return;
  const int hh = e >> 12, rem = e & 4095;
  const int tile = rem >> 10, lane = (rem >> 4) & 63, r = rem & 15;
  const int row = (tile >> 1) * 32 + acc_row(r, lane >> 5), col = (tile & 1) * 32 + (lane & 31);
  auto val = [&](int q, int key) {
    if (key >= WA_N) return -INFINITY;
    if (q >= WA_N) return 0.f;
    return rpb[rpb_index<7>(q, key) * heads + hh];
  };
  if (biasT) biasT[e] = val(col, row);
  if (biasN) biasN[e] = val(row, col);
}

// sums[h][t] (column sums over windows of partial[win][h][T + 2*HD]) ->
// d_rpb_table[t][h], dk_pad / dv_pad [h*HD + d]
template <int WS, int HD>
__global__ void winattn_bwd_scatter(const float* __restrict__ sums, int heads, float* d_rpb, float* dk_pad,
                                    float* dv_pad, float* dq_pad) {
  constexpr int T = (2 * WS - 1) * (2 * WS - 1), R = T + 2 * HD;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= heads * R) return;
  const int h = e / R, t = e % R;
  const float s = sums[e];
  if (t < T) d_rpb[t * heads + h] = s;
  else if (t < T + HD) { if (dk_pad) dk_pad[h * HD + t - T] = s; }
  else if (dv_pad) dv_pad[h * HD + t - T - HD] = s;
  if (dq_pad && t < HD) dq_pad[h * HD + t] = 0.f;  // pad queries never receive gradient
}

static int make_params(const mdemi_winattn_desc* d, WinParams& p, int& nwin) {
  MDEMI_REQUIRE(d, "winattn: null descriptor");
  MDEMI_REQUIRE(d->B > 0 && d->H > 0 && d->W > 0 && d->heads > 0, "winattn: bad sizes");
  MDEMI_REQUIRE(d->window == 7 && d->head_dim == 32, "winattn: only window 7 / head_dim 32 are built (got %d/%d)",
                d->window, d->head_dim);
  MDEMI_REQUIRE(d->shift >= 0 && d->shift < d->window, "winattn: bad shift %d", d->shift);
  MDEMI_REQUIRE(d->q && d->k && d->v && d->rpb_table, "winattn: null input");
  MDEMI_REQUIRE(d->qk_ld % 4 == 0 && d->v_ld % 4 == 0 && d->out_ld % 4 == 0, "winattn: row strides must be %% 4");
  const int ws = d->window;
  p.g.B = d->B; p.g.H = d->H; p.g.W = d->W;
  p.g.Hp = (d->H + ws - 1) / ws * ws; p.g.Wp = (d->W + ws - 1) / ws * ws;
  p.g.nWh = p.g.Hp / ws; p.g.nWw = p.g.Wp / ws;
  p.g.shift = d->shift; p.g.heads = d->heads;
  p.scale = d->scale;
  p.q = d->q; p.k = d->k; p.qk_ld = d->qk_ld; p.q_pad = d->q_pad; p.k_pad = d->k_pad;
  p.v = d->v; p.v_ld = d->v_ld; p.v_pad = d->v_pad;
  p.rpb = d->rpb_table;
  p.out = d->out; p.out_ld = d->out_ld;
  p.lse = d->lse;
  p.dout = d->dout; p.dq = d->dq; p.dk = d->dk; p.dqk_ld = d->dqk_ld; p.dv = d->dv; p.dv_ld = d->dv_ld;
  p.partial = (float*)d->workspace;
  {
    const int64_t rows = (int64_t)d->B * d->H * d->W;
    const int64_t lds[4] = {d->qk_ld, d->out_ld, d->dqk_ld, d->dv_ld};
    bool ok = rows < (1 << 24);
    for (int64_t ld : lds) ok = ok && ld >= 0 && ld < (1 << 24) && rows * ld < (int64_t(1) << 32);
    p.off32 = ok;
  }
  nwin = d->B * p.g.nWh * p.g.nWw;
  return MDEMI_OK;
}

}  // namespace mdemi

using namespace mdemi;

static int wa_items(const mdemi_winattn_desc* d, int nwin) { return nwin * d->heads; }
static size_t wa_bias_bytes(const mdemi_winattn_desc* d) { return (size_t)d->heads * 4096 * sizeof(float); }

extern "C" size_t mdemi_winattn_fwd_workspace_size(const mdemi_winattn_desc* d) {
  WinParams p;
  int nwin;
  if (make_params(d, p, nwin)) return 0;
  return wa_bias_bytes(d);
}

extern "C" int mdemi_winattn_fwd(const mdemi_winattn_desc* d, void* stream) {
  WinParams p;
  int nwin;
  int rc = make_params(d, p, nwin);
  if (rc) return rc;
  MDEMI_REQUIRE(d->out, "winattn_fwd: null out");
  if (!d->workspace || (size_t)d->workspace_bytes < wa_bias_bytes(d)) {
    set_error("winattn_fwd: needs %zu workspace bytes", wa_bias_bytes(d));
    return MDEMI_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  float* biasT = (float*)d->workspace;
  hipLaunchKernelGGL(wa_bias_kernel, dim3(d->heads * 16), dim3(256), 0, st, d->rpb_table, d->heads, biasT,
                     (float*)nullptr);
  const int nitems = wa_items(d, nwin);
  hipLaunchKernelGGL((winattn_fwd_kernel<7, 32>), dim3(cdiv(nitems, WA_WAVES)), dim3(64 * WA_WAVES), 0, st, p,
                     (const float*)biasT, nitems);
  return check_launch("winattn_fwd");
}

// workspace: [partials items x R | bias T | sums heads*R | colsum scratch]
static size_t wa_part_bytes(int items, int R) { return align_up((size_t)items * R * 4, 256); }
extern "C" size_t mdemi_winattn_bwd_workspace_size(const mdemi_winattn_desc* d) {
  WinParams p;
  int nwin;
  if (make_params(d, p, nwin)) return 0;
  const int R = WA_T + 2 * WA_HD;
  const int items = wa_items(d, nwin);
  return wa_part_bytes(items, R) + wa_bias_bytes(d) + align_up((size_t)d->heads * R * 4, 256) +
         colsum_ws_bytes(nwin, (int64_t)d->heads * R);
}

extern "C" int mdemi_winattn_bwd(const mdemi_winattn_desc* d, void* stream) {
  return mdemi_winattn_bwd_bias(d, nullptr, stream);
}

extern "C" int mdemi_winattn_bwd_bias(const mdemi_winattn_desc* d, const float* bias_expanded, void* stream) {
  WinParams p;
  int nwin;
  int rc = make_params(d, p, nwin);
  if (rc) return rc;
  MDEMI_REQUIRE(d->dout && d->dq && d->dk && d->dv && d->d_rpb_table, "winattn_bwd: null gradient buffer");
  MDEMI_REQUIRE(d->out && d->lse, "winattn_bwd: needs the forward output and its saved lse");
  MDEMI_REQUIRE(d->dqk_ld % 4 == 0 && d->dv_ld % 4 == 0, "winattn_bwd: gradient strides must be %% 4");
  const size_t need = mdemi_winattn_bwd_workspace_size(d);
  if (!d->workspace || (size_t)d->workspace_bytes < need) {
    set_error("winattn_bwd: needs %zu workspace bytes", need);
    return MDEMI_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const int R = WA_T + 2 * WA_HD;
  const int items = wa_items(d, nwin);
  char* ws = (char*)d->workspace;
  p.partial = (float*)ws;
  float* biasT = (float*)(ws + wa_part_bytes(items, R));
  float* sums = (float*)((char*)biasT + wa_bias_bytes(d));
  void* cws = (char*)sums + align_up((size_t)d->heads * R * 4, 256);
  if (bias_expanded)  // the forward's expansion of the same table (mdemi_winattn_fwd's workspace)
    biasT = const_cast<float*>(bias_expanded);
  else
    hipLaunchKernelGGL(wa_bias_kernel, dim3(d->heads * 16), dim3(256), 0, st, d->rpb_table, d->heads, biasT,
                       (float*)nullptr);
  hipLaunchKernelGGL((winattn_bwd_kernel<7, 32>), dim3((unsigned)cdiv(items, WA_WAVES)), dim3(64 * WA_WAVES), 0, st,
                     p, (const float*)biasT, items);
  int rc2 = colsum_launch(p.partial, nwin, (int64_t)d->heads * R, (int64_t)d->heads * R, sums, 0, cws, st);
  if (rc2) return rc2;
  hipLaunchKernelGGL((winattn_bwd_scatter<7, 32>), dim3((d->heads * R + 255) / 256), dim3(256), 0, st, sums, d->heads,
                     d->d_rpb_table, d->dk_pad, d->dv_pad, d->dq_pad);
  return check_launch("winattn_bwd");
}
