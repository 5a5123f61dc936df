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
  float* partial;  // [nwin][heads][T + 2*HD]
  float* dsum;     // [nwin][heads][N]  D_i = dO_i . O_i
};

template <int WS, int HD>
__global__ __launch_bounds__(64) void winattn_fwd_kernel(WinParams p) {
  constexpr int N = WS * WS, T = (2 * WS - 1) * (2 * WS - 1), H4 = HD / 4;
  static_assert(N <= 64, "window too large for one wave");
  __shared__ float4 Ks[N][H4];
  __shared__ float4 Vs[N][H4];
  __shared__ float tab[T];
  const WinGeom& g = p.g;
  const int win = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const Win<WS> w(g, win);
  for (int e = lane; e < N * H4; e += 64) {
    const int j = e / H4, q4 = e % H4;
    const int r = w.row(g, j);
    Ks[j][q4] = ld_tok4(p.k, p.qk_ld, r, p.k_pad, h * HD + 4 * q4);
    Vs[j][q4] = ld_tok4(p.v, p.v_ld, r, p.v_pad, h * HD + 4 * q4);
  }
  for (int e = lane; e < T; e += 64) tab[e] = p.rpb[e * g.heads + h];
  __syncthreads();
  const int i = lane;
  if (i >= N) return;
  const int ri = w.row(g, i);
  float* lse_row = p.lse ? p.lse + ((int64_t)win * g.heads + h) * N : nullptr;
  if (ri < 0) {  // pad query: its output is cropped away
    if (lse_row) lse_row[i] = INFINITY;
    return;
  }
  const int reg_i = g.shift > 0 ? w.region(g, i) : 0;
  float4 q[H4];
  load_row<HD>(q, p.q + (int64_t)ri * p.qk_ld + h * HD);
#pragma unroll
  for (int c = 0; c < H4; ++c) { q[c].x *= p.scale; q[c].y *= p.scale; q[c].z *= p.scale; q[c].w *= p.scale; }
  float s[N];
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < H4; ++c) acc += dot4(q[c], Ks[j][c]);
    acc += tab[rpb_index<WS>(i, j)];
    if (g.shift > 0 && w.region(g, j) != reg_i) acc += -100.f;
    s[j] = acc;
    m = fmaxf(m, acc);
  }
  float l = 0.f;
#pragma unroll
  for (int j = 0; j < N; ++j) { s[j] = __expf(s[j] - m); l += s[j]; }
  const float inv = 1.f / l;
  if (lse_row) lse_row[i] = m + __logf(l);
  float4 o[H4];
#pragma unroll
  for (int c = 0; c < H4; ++c) o[c] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const float pj = s[j] * inv;
#pragma unroll
    for (int c = 0; c < H4; ++c) {
      const float4 v = Vs[j][c];
      o[c].x = fmaf(pj, v.x, o[c].x); o[c].y = fmaf(pj, v.y, o[c].y);
      o[c].z = fmaf(pj, v.z, o[c].z); o[c].w = fmaf(pj, v.w, o[c].w);
    }
  }
  float4* dst = reinterpret_cast<float4*>(p.out + (int64_t)ri * p.out_ld + h * HD);
#pragma unroll
  for (int c = 0; c < H4; ++c) dst[c] = o[c];
}

// Backward, split by role so each kernel stages only 2 row-sets in LDS
// (~13 KB: ~3 waves/SIMD instead of 1) and keeps no score matrix:
//   P_ij = exp(S_ij - lse_i) from the forward's saved log-sum-exp,
//   D_i = dO_i . O_i (the identity rowsum(P o dP) = dO . O), dS = P (dP - D).
// Q-kernel (lane = query i, K/V rows in LDS): dQ_i = scale * sum_j dS_ij k_j,
//   bias-table gradient through LDS atomics, D_i for the KV-kernel.
// KV-kernel (lane = key j, scale*Q / dO rows in LDS): dK_j = sum_i dS_ij (scale q_i),
//   dV_j = sum_i P_ij dO_i; pad keys add into per-window pad sums.
template <int WS, int HD>
__global__ __launch_bounds__(64) void winattn_bwd_q_kernel(WinParams p) {
  constexpr int N = WS * WS, T = (2 * WS - 1) * (2 * WS - 1), H4 = HD / 4;
  __shared__ float4 Ks[N][H4];
  __shared__ float4 Vs[N][H4];
  __shared__ float tab[T];
  __shared__ float tabg[T];
  const WinGeom& g = p.g;
  const int win = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const Win<WS> w(g, win);
  for (int e = lane; e < N * H4; e += 64) {
    const int j = e / H4, q4 = e % H4;
    const int r = w.row(g, j);
    Ks[j][q4] = ld_tok4(p.k, p.qk_ld, r, p.k_pad, h * HD + 4 * q4);
    Vs[j][q4] = ld_tok4(p.v, p.v_ld, r, p.v_pad, h * HD + 4 * q4);
  }
  for (int e = lane; e < T; e += 64) { tab[e] = p.rpb[e * g.heads + h]; tabg[e] = 0.f; }
  __syncthreads();
  const int i = lane;
  const int64_t rowbase = ((int64_t)win * g.heads + h) * N;
  if (i < N) {
    const int ri = w.row(g, i);
    if (ri >= 0) {
      const int reg_i = g.shift > 0 ? w.region(g, i) : 0;
      float4 q[H4], dO[H4];
      load_row<HD>(q, p.q + (int64_t)ri * p.qk_ld + h * HD);
      load_row<HD>(dO, p.dout + (int64_t)ri * p.out_ld + h * HD);
      float D = 0.f;
      {
        float4 o[H4];
        load_row<HD>(o, p.out + (int64_t)ri * p.out_ld + h * HD);
#pragma unroll
        for (int c = 0; c < H4; ++c) {
          D += dot4(dO[c], o[c]);
          q[c].x *= p.scale; q[c].y *= p.scale; q[c].z *= p.scale; q[c].w *= p.scale;
        }
      }
      const float lse = p.lse[rowbase + i];
      float4 dq[H4];
#pragma unroll
      for (int c = 0; c < H4; ++c) dq[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int j = 0; j < N; ++j) {
        float s = 0.f, dp = 0.f;
#pragma unroll
        for (int c = 0; c < H4; ++c) { s += dot4(q[c], Ks[j][c]); dp += dot4(dO[c], Vs[j][c]); }
        s += tab[rpb_index<WS>(i, j)];
        if (g.shift > 0 && w.region(g, j) != reg_i) s += -100.f;
        const float ds = __expf(s - lse) * (dp - D);
        atomicAdd(&tabg[rpb_index<WS>(i, j)], ds);
#pragma unroll
        for (int c = 0; c < H4; ++c) {
          const float4 kk = Ks[j][c];
          dq[c].x = fmaf(ds, kk.x, dq[c].x); dq[c].y = fmaf(ds, kk.y, dq[c].y);
          dq[c].z = fmaf(ds, kk.z, dq[c].z); dq[c].w = fmaf(ds, kk.w, dq[c].w);
        }
      }
      float4* dst = reinterpret_cast<float4*>(p.dq + (int64_t)ri * p.dqk_ld + h * HD);
#pragma unroll
      for (int c = 0; c < H4; ++c)
        dst[c] = make_float4(dq[c].x * p.scale, dq[c].y * p.scale, dq[c].z * p.scale, dq[c].w * p.scale);
      p.dsum[rowbase + i] = D;
    } else {
      p.dsum[rowbase + i] = 0.f;
    }
  }
  __syncthreads();
  float* P = p.partial + ((int64_t)win * g.heads + h) * (T + 2 * HD);
  for (int e = lane; e < T; e += 64) P[e] = tabg[e];
}

template <int WS, int HD>
__global__ __launch_bounds__(64) void winattn_bwd_kv_kernel(WinParams p) {
  constexpr int N = WS * WS, T = (2 * WS - 1) * (2 * WS - 1), H4 = HD / 4;
  __shared__ float4 Qs[N][H4];  // scale * q
  __shared__ float4 Ds[N][H4];  // dO
  __shared__ float tab[T];
  __shared__ float lse_s[N], D_s[N];
  __shared__ int reg_s[N];
  __shared__ float padk[HD], padv[HD];
  const WinGeom& g = p.g;
  const int win = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const Win<WS> w(g, win);
  const int64_t rowbase = ((int64_t)win * g.heads + h) * N;
  for (int e = lane; e < N * H4; e += 64) {
    const int i = e / H4, q4 = e % H4;
    const int r = w.row(g, i);
    float4 qq = ld_tok4(p.q, p.qk_ld, r, p.q_pad, h * HD + 4 * q4);
    qq.x *= p.scale; qq.y *= p.scale; qq.z *= p.scale; qq.w *= p.scale;
    Qs[i][q4] = qq;
    Ds[i][q4] = r >= 0 ? *reinterpret_cast<const float4*>(p.dout + (int64_t)r * p.out_ld + h * HD + 4 * q4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int e = lane; e < T; e += 64) tab[e] = p.rpb[e * g.heads + h];
  if (lane < N) {
    lse_s[lane] = p.lse[rowbase + lane];  // +inf for pad queries -> P = 0
    D_s[lane] = p.dsum[rowbase + lane];
    reg_s[lane] = g.shift > 0 ? w.region(g, lane) : 0;
  }
  if (lane < HD) { padk[lane] = 0.f; padv[lane] = 0.f; }
  __syncthreads();
  const int j = lane;
  if (j < N) {
    const int rj = w.row(g, j);
    const int reg_j = reg_s[j];
    float4 kj[H4], vj[H4], dk[H4], dv[H4];
#pragma unroll
    for (int c = 0; c < H4; ++c) {
      kj[c] = ld_tok4(p.k, p.qk_ld, rj, p.k_pad, h * HD + 4 * c);
      vj[c] = ld_tok4(p.v, p.v_ld, rj, p.v_pad, h * HD + 4 * c);
      dk[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      dv[c] = dk[c];
    }
    for (int i = 0; i < N; ++i) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int c = 0; c < H4; ++c) { s += dot4(Qs[i][c], kj[c]); dp += dot4(Ds[i][c], vj[c]); }
      s += tab[rpb_index<WS>(i, j)];
      if (g.shift > 0 && reg_s[i] != reg_j) s += -100.f;
      const float pr = __expf(s - lse_s[i]);
      const float ds = pr * (dp - D_s[i]);
#pragma unroll
      for (int c = 0; c < H4; ++c) {
        const float4 qq = Qs[i][c], dd = Ds[i][c];
        dk[c].x = fmaf(ds, qq.x, dk[c].x); dk[c].y = fmaf(ds, qq.y, dk[c].y);
        dk[c].z = fmaf(ds, qq.z, dk[c].z); dk[c].w = fmaf(ds, qq.w, dk[c].w);
        dv[c].x = fmaf(pr, dd.x, dv[c].x); dv[c].y = fmaf(pr, dd.y, dv[c].y);
        dv[c].z = fmaf(pr, dd.z, dv[c].z); dv[c].w = fmaf(pr, dd.w, dv[c].w);
      }
    }
    if (rj >= 0) {
      float4* dkd = reinterpret_cast<float4*>(p.dk + (int64_t)rj * p.dqk_ld + h * HD);
      float4* dvd = reinterpret_cast<float4*>(p.dv + (int64_t)rj * p.dv_ld + h * HD);
#pragma unroll
      for (int c = 0; c < H4; ++c) { dkd[c] = dk[c]; dvd[c] = dv[c]; }
    } else {
#pragma unroll
      for (int c = 0; c < H4; ++c) {
        atomicAdd(&padk[4 * c + 0], dk[c].x); atomicAdd(&padk[4 * c + 1], dk[c].y);
        atomicAdd(&padk[4 * c + 2], dk[c].z); atomicAdd(&padk[4 * c + 3], dk[c].w);
        atomicAdd(&padv[4 * c + 0], dv[c].x); atomicAdd(&padv[4 * c + 1], dv[c].y);
        atomicAdd(&padv[4 * c + 2], dv[c].z); atomicAdd(&padv[4 * c + 3], dv[c].w);
      }
    }
  }
  __syncthreads();
  float* P = p.partial + ((int64_t)win * g.heads + h) * (T + 2 * HD);
  if (lane < HD) { P[T + lane] = padk[lane]; P[T + HD + lane] = padv[lane]; }
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
  nwin = d->B * p.g.nWh * p.g.nWw;
  return MDEMI_OK;
}

}  // namespace mdemi

using namespace mdemi;

extern "C" int mdemi_winattn_fwd(const mdemi_winattn_desc* d, void* stream) {
  WinParams p;
  int nwin;
  int rc = make_params(d, p, nwin);
  if (rc) return rc;
  MDEMI_REQUIRE(d->out, "winattn_fwd: null out");
  hipLaunchKernelGGL((winattn_fwd_kernel<7, 32>), dim3(nwin, d->heads), dim3(64), 0, (hipStream_t)stream, p);
  return check_launch("winattn_fwd");
}

// workspace: [partials nwin x heads*R | D nwin x heads x N | sums heads*R | colsum scratch]
static size_t wa_part_bytes(int nwin, int heads, int R) { return align_up((size_t)nwin * heads * R * 4, 256); }
static size_t wa_dsum_bytes(int nwin, int heads, int N) { return align_up((size_t)nwin * heads * N * 4, 256); }
extern "C" size_t mdemi_winattn_bwd_workspace_size(const mdemi_winattn_desc* d) {
  WinParams p;
  int nwin;
  if (make_params(d, p, nwin)) return 0;
  const int R = (2 * d->window - 1) * (2 * d->window - 1) + 2 * d->head_dim;
  return wa_part_bytes(nwin, d->heads, R) + wa_dsum_bytes(nwin, d->heads, d->window * d->window) +
         align_up((size_t)d->heads * R * 4, 256) + colsum_ws_bytes(nwin, (int64_t)d->heads * R);
}

extern "C" int mdemi_winattn_bwd(const mdemi_winattn_desc* d, void* stream) {
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
  const int R = 13 * 13 + 64;
  p.dsum = (float*)((char*)d->workspace + wa_part_bytes(nwin, d->heads, R));
  hipLaunchKernelGGL((winattn_bwd_q_kernel<7, 32>), dim3(nwin, d->heads), dim3(64), 0, st, p);
  hipLaunchKernelGGL((winattn_bwd_kv_kernel<7, 32>), dim3(nwin, d->heads), dim3(64), 0, st, p);
  float* sums = (float*)((char*)p.dsum + wa_dsum_bytes(nwin, d->heads, 49));
  void* cws = (char*)sums + align_up((size_t)d->heads * R * 4, 256);
  int rc2 = colsum_launch(p.partial, nwin, (int64_t)d->heads * R, (int64_t)d->heads * R, sums, 0, cws, st);
  if (rc2) return rc2;
  hipLaunchKernelGGL((winattn_bwd_scatter<7, 32>), dim3((d->heads * R + 255) / 256), dim3(256), 0, st, sums, d->heads,
                     d->d_rpb_table, d->dk_pad, d->dv_pad, d->dq_pad);
  return check_launch("winattn_bwd");
}
