// EfficientNet-B5 (tf_efficientnet_b5_ap) encoder ops over NHWC activations:
// the depthwise conv of every MBConv / DepthwiseSeparable block, the
// SqueezeExcite pooling + gate MLP + channel scaling, and the padded image
// layout for conv_stem.  The encoder is third-party in the reference
// (torch.hub 'rwightman/gen-efficientnet-pytorch', unet_adaptive_bins.py:129,
// depthformer_v8.py:89; its modules are walked at unet_adaptive_bins.py:65-73);
// everything here restates that published architecture.  All of it is
// HBM-bound: each kernel streams its activation once and keeps the small
// per-channel state (KxK taps, gates) in registers.
#include "common.h"
#include "mdemi_ext.h"

namespace mdemi {

static unsigned grid_1d(int64_t total, int per_block = 256) {
  int64_t g = cdiv(total, per_block);
  return (unsigned)(g < 1 ? 1 : (g > 65535 * 8 ? 65535 * 8 : g));
}

// ---------------------------------------------------------------------------
// depthwise conv forward: thread = (n, oy, TX consecutive ox, 4 channels).
// The TX outputs share one sweep over the (TX-1)*S+K input columns of each
// kernel row, so every input quad is fetched once per kernel row.
// ---------------------------------------------------------------------------
template <int K, int S, int TX>
__global__ __launch_bounds__(256) void dwconv_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         float* __restrict__ y, int N, int H, int W, int C, int pad_t,
                                                         int pad_l, int OH, int OW) {
  constexpr int KK = K * K, SPAN = (TX - 1) * S + K;
  const int C4 = C >> 2, OWT = (OW + TX - 1) / TX;
  const int64_t total = (int64_t)N * OH * OWT * C4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    int64_t t = e / C4;
    const int oxt = (int)(t % OWT); t /= OWT;
    const int oy = (int)(t % OH);
    const int n = (int)(t / OH);
    const int c = c4 * 4;
    const int ox0 = oxt * TX;
    const int ix0 = ox0 * S - pad_l;
    float4 acc[TX];
#pragma unroll
    for (int q = 0; q < TX; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* w0 = w + (int64_t)c * KK;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy * S - pad_t + ky;
      if (iy < 0 || iy >= H) continue;
      float4 wk[K];
#pragma unroll
      for (int kx = 0; kx < K; ++kx)
        wk[kx] = make_float4(w0[ky * K + kx], w0[KK + ky * K + kx], w0[2 * KK + ky * K + kx],
                             w0[3 * KK + ky * K + kx]);
      const float* row = x + (((int64_t)n * H + iy) * W) * C + c;
#pragma unroll
      for (int j = 0; j < SPAN; ++j) {
        const int ix = ix0 + j;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ix >= 0 && ix < W) v = *reinterpret_cast<const float4*>(row + (int64_t)ix * C);
#pragma unroll
        for (int q = 0; q < TX; ++q) {
          const int kx = j - q * S;
          if (kx >= 0 && kx < K) {
            acc[q].x = fmaf(v.x, wk[kx].x, acc[q].x);
            acc[q].y = fmaf(v.y, wk[kx].y, acc[q].y);
            acc[q].z = fmaf(v.z, wk[kx].z, acc[q].z);
            acc[q].w = fmaf(v.w, wk[kx].w, acc[q].w);
          }
        }
      }
    }
    float* out = y + (((int64_t)n * OH + oy) * OW) * C + c;
#pragma unroll
    for (int q = 0; q < TX; ++q)
      if (ox0 + q < OW) *reinterpret_cast<float4*>(out + (int64_t)(ox0 + q) * C) = acc[q];
  }
}

// depthwise conv input gradient, a gather: dx[iy][ix] = sum over taps of
// dy[oy][ox] * w[ky][kx] with oy*S = iy + pad_t - ky, ox*S = ix + pad_l - kx.
template <int K, int S, int TX>
__global__ __launch_bounds__(256) void dwconv_dx_kernel(const float* __restrict__ dy, const float* __restrict__ w,
                                                        float* __restrict__ dx, int N, int H, int W, int C, int pad_t,
                                                        int pad_l, int OH, int OW) {
  constexpr int KK = K * K;
  const int C4 = C >> 2, WT = (W + TX - 1) / TX;
  const int64_t total = (int64_t)N * H * WT * C4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    int64_t t = e / C4;
    const int ixt = (int)(t % WT); t /= WT;
    const int iy = (int)(t % H);
    const int n = (int)(t / H);
    const int c = c4 * 4;
    const int ix0 = ixt * TX;
    float4 acc[TX];
#pragma unroll
    for (int q = 0; q < TX; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* w0 = w + (int64_t)c * KK;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int ny = iy + pad_t - ky;
      if (ny < 0 || (S > 1 && (ny % S) != 0)) continue;
      const int oy = ny / S;
      if (oy >= OH) continue;
      const float* row = dy + (((int64_t)n * OH + oy) * OW) * C + c;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const float4 wk = make_float4(w0[ky * K + kx], w0[KK + ky * K + kx], w0[2 * KK + ky * K + kx],
                                      w0[3 * KK + ky * K + kx]);
#pragma unroll
        for (int q = 0; q < TX; ++q) {
          const int nx = ix0 + q + pad_l - kx;
          if (nx < 0 || (S > 1 && (nx % S) != 0)) continue;
          const int ox = nx / S;
          if (ox >= OW) continue;
          const float4 v = *reinterpret_cast<const float4*>(row + (int64_t)ox * C);
          acc[q].x = fmaf(v.x, wk.x, acc[q].x);
          acc[q].y = fmaf(v.y, wk.y, acc[q].y);
          acc[q].z = fmaf(v.z, wk.z, acc[q].z);
          acc[q].w = fmaf(v.w, wk.w, acc[q].w);
        }
      }
    }
    float* out = dx + (((int64_t)n * H + iy) * W) * C + c;
#pragma unroll
    for (int q = 0; q < TX; ++q)
      if (ix0 + q < W) *reinterpret_cast<float4*>(out + (int64_t)(ix0 + q) * C) = acc[q];
  }
}

// stride-1 input gradient as a row sweep (the correlation of dy with the
// flipped taps): the TX outputs of a thread share one pass over the TX+K-1
// dy columns of each tap row, instead of K*K*TX separate loads.
template <int K, int TX>
__global__ __launch_bounds__(256) void dwconv_dx_s1_kernel(const float* __restrict__ dy, const float* __restrict__ w,
                                                           float* __restrict__ dx, int N, int H, int W, int C,
                                                           int pad_t, int pad_l, int OH, int OW) {
  constexpr int KK = K * K, SPAN = TX + K - 1;
  const int C4 = C >> 2, WT = (W + TX - 1) / TX;
  const int64_t total = (int64_t)N * H * WT * C4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    int64_t t = e / C4;
    const int ixt = (int)(t % WT); t /= WT;
    const int iy = (int)(t % H);
    const int n = (int)(t / H);
    const int c = c4 * 4;
    const int ix0 = ixt * TX;
    // output columns ox = ix + pad_l - kx; the sweep starts at ix0 + pad_l - (K-1)
    const int ox0 = ix0 + pad_l - (K - 1);
    float4 acc[TX];
#pragma unroll
    for (int q = 0; q < TX; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* w0 = w + (int64_t)c * KK;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int oy = iy + pad_t - ky;
      if (oy < 0 || oy >= OH) continue;
      float4 wk[K];
#pragma unroll
      for (int kx = 0; kx < K; ++kx)
        wk[kx] = make_float4(w0[ky * K + kx], w0[KK + ky * K + kx], w0[2 * KK + ky * K + kx],
                             w0[3 * KK + ky * K + kx]);
      const float* row = dy + (((int64_t)n * OH + oy) * OW) * C + c;
#pragma unroll
      for (int j = 0; j < SPAN; ++j) {
        const int ox = ox0 + j;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ox >= 0 && ox < OW) v = *reinterpret_cast<const float4*>(row + (int64_t)ox * C);
#pragma unroll
        for (int q = 0; q < TX; ++q) {
          const int kx = q + (K - 1) - j;  // ox = ix0 + q + pad_l - kx
          if (kx >= 0 && kx < K) {
            acc[q].x = fmaf(v.x, wk[kx].x, acc[q].x);
            acc[q].y = fmaf(v.y, wk[kx].y, acc[q].y);
            acc[q].z = fmaf(v.z, wk[kx].z, acc[q].z);
            acc[q].w = fmaf(v.w, wk[kx].w, acc[q].w);
          }
        }
      }
    }
    float* out = dx + (((int64_t)n * H + iy) * W) * C + c;
#pragma unroll
    for (int q = 0; q < TX; ++q)
      if (ix0 + q < W) *reinterpret_cast<float4*>(out + (int64_t)(ix0 + q) * C) = acc[q];
  }
}

// depthwise conv weight gradient: block = 64 channel quads x 4 pixel lanes over
// one chunk of output pixels; K*K quad accumulators per thread; the 4 pixel
// lanes are combined through LDS and each (chunk, channel, tap) partial is
// written to part[chunk][c*KK + tap] for a deterministic column sum.
template <int K, int S>
__global__ __launch_bounds__(256) void dwconv_dw_partial(const float* __restrict__ dy, const float* __restrict__ x,
                                                         float* __restrict__ part, int N, int H, int W, int C,
                                                         int pad_t, int pad_l, int OH, int OW, int64_t pix_per_chunk) {
  constexpr int KK = K * K;
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int C4 = C >> 2;
  const int c4 = blockIdx.x * 64 + lane;
  const bool cok = c4 < C4;
  const int c = (cok ? c4 : 0) * 4;
  const int64_t npix = (int64_t)N * OH * OW;
  const int64_t p0 = (int64_t)blockIdx.y * pix_per_chunk;
  const int64_t p1 = min(npix, p0 + pix_per_chunk);
  float4 acc[KK];
#pragma unroll
  for (int k = 0; k < KK; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (cok) {
    for (int64_t p = p0 + ty; p < p1; p += 4) {
      const int ox = (int)(p % OW);
      const int64_t t = p / OW;
      const int oy = (int)(t % OH);
      const int n = (int)(t / OH);
      const float4 g = *reinterpret_cast<const float4*>(dy + p * C + c);
      const float* xb = x + ((int64_t)n * H * W) * C + c;
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        const int iy = oy * S - pad_t + ky;
        if (iy < 0 || iy >= H) continue;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int ix = ox * S - pad_l + kx;
          if (ix < 0 || ix >= W) continue;
          const float4 v = *reinterpret_cast<const float4*>(xb + ((int64_t)iy * W + ix) * C);
          float4& a = acc[ky * K + kx];
          a.x = fmaf(g.x, v.x, a.x);
          a.y = fmaf(g.y, v.y, a.y);
          a.z = fmaf(g.z, v.z, a.z);
          a.w = fmaf(g.w, v.w, a.w);
        }
      }
    }
  }
  float* dst = part + (int64_t)blockIdx.y * C * KK;
#pragma unroll
  for (int k = 0; k < KK; ++k) {
    red[ty][lane] = acc[k];
    __syncthreads();
    if (ty == 0 && cok) {
      float4 s = red[0][lane];
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const float4 v = red[q][lane];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      dst[(int64_t)(c + 0) * KK + k] = s.x;
      dst[(int64_t)(c + 1) * KK + k] = s.y;
      dst[(int64_t)(c + 2) * KK + k] = s.z;
      dst[(int64_t)(c + 3) * KK + k] = s.w;
    }
    __syncthreads();
  }
}

// stride-1 weight gradient with a row sweep: a work item is TX consecutive
// output columns of one row; per tap row it loads the TX+K-1 input quads once
// and the TX dy quads, and updates all K*K tap accumulators.
template <int K, int TX>
__global__ __launch_bounds__(256) void dwconv_dw_partial_s1(const float* __restrict__ dy, const float* __restrict__ x,
                                                            float* __restrict__ part, int N, int H, int W, int C,
                                                            int pad_t, int pad_l, int OH, int OW,
                                                            int64_t grp_per_chunk) {
  constexpr int KK = K * K, SPAN = TX + K - 1;
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int C4 = C >> 2;
  const int c4 = blockIdx.x * 64 + lane;
  const bool cok = c4 < C4;
  const int c = (cok ? c4 : 0) * 4;
  const int OWT = (OW + TX - 1) / TX;
  const int64_t ngrp = (int64_t)N * OH * OWT;
  const int64_t g0 = (int64_t)blockIdx.y * grp_per_chunk;
  const int64_t g1 = min(ngrp, g0 + grp_per_chunk);
  float4 acc[KK];
#pragma unroll
  for (int k = 0; k < KK; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (cok) {
    for (int64_t gi = g0 + ty; gi < g1; gi += 4) {
      const int oxt = (int)(gi % OWT);
      const int64_t t = gi / OWT;
      const int oy = (int)(t % OH);
      const int n = (int)(t / OH);
      const int ox0 = oxt * TX;
      float4 g[TX];
#pragma unroll
      for (int q = 0; q < TX; ++q) {
        g[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ox0 + q < OW) g[q] = *reinterpret_cast<const float4*>(dy + (((int64_t)n * OH + oy) * OW + ox0 + q) * C + c);
      }
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        const int iy = oy - pad_t + ky;
        if (iy < 0 || iy >= H) continue;
        const float* row = x + (((int64_t)n * H + iy) * W) * C + c;
#pragma unroll
        for (int j = 0; j < SPAN; ++j) {
          const int ix = ox0 - pad_l + j;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (ix >= 0 && ix < W) v = *reinterpret_cast<const float4*>(row + (int64_t)ix * C);
#pragma unroll
          for (int q = 0; q < TX; ++q) {
            const int kx = j - q;
            if (kx >= 0 && kx < K) {
              float4& a = acc[ky * K + kx];
              a.x = fmaf(g[q].x, v.x, a.x);
              a.y = fmaf(g[q].y, v.y, a.y);
              a.z = fmaf(g[q].z, v.z, a.z);
              a.w = fmaf(g[q].w, v.w, a.w);
            }
          }
        }
      }
    }
  }
  float* dst = part + (int64_t)blockIdx.y * C * KK;
#pragma unroll
  for (int k = 0; k < KK; ++k) {
    red[ty][lane] = acc[k];
    __syncthreads();
    if (ty == 0 && cok) {
      float4 sum = red[0][lane];
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const float4 v = red[q][lane];
        sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
      }
      dst[(int64_t)(c + 0) * KK + k] = sum.x;
      dst[(int64_t)(c + 1) * KK + k] = sum.y;
      dst[(int64_t)(c + 2) * KK + k] = sum.z;
      dst[(int64_t)(c + 3) * KK + k] = sum.w;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Stride-1 depthwise conv as TY x TX output blocks per thread (35 of the 39 MBConv blocks).
// A block's TY + K - 1 input rows are each fetched once (SPAN = TX + K - 1 quads) and feed
// every output row they touch, with all K*K taps of the thread's 4 channels in registers:
// (TY+K-1)*SPAN / (TY*TX) quad loads per output quad, against K*SPAN / TX for one output row
// (K 5: 4 vs 10).  The one-row kernels re-fetched each input row K times through L1/L2 and
// ran at 1.2 TB/s (K 5) / 2.8 TB/s (K 3) on the configs[4] shapes (profiles/round6/).  Taps
// accumulate in the same order as dwconv_fwd_kernel (ky ascending, then kx): bit-identical.
// ---------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ void dw_load_taps(const float* __restrict__ w, int c, float4 (&wk)[K][K]) {
  constexpr int KK = K * K;
  const float* w0 = w + (int64_t)c * KK;
#pragma unroll
  for (int ky = 0; ky < K; ++ky)
#pragma unroll
    for (int kx = 0; kx < K; ++kx)
      wk[ky][kx] = make_float4(w0[ky * K + kx], w0[KK + ky * K + kx], w0[2 * KK + ky * K + kx],
                               w0[3 * KK + ky * K + kx]);
}

__device__ __forceinline__ void fma4(float4& a, const float4& v, const float4& w) {
  a.x = fmaf(v.x, w.x, a.x);
  a.y = fmaf(v.y, w.y, a.y);
  a.z = fmaf(v.z, w.z, a.z);
  a.w = fmaf(v.w, w.w, a.w);
}

template <int K, int TX, int TY>
__global__ __launch_bounds__(256) void dwconv_fwd_s1_blk(const float* __restrict__ x, const float* __restrict__ w,
                                                         float* __restrict__ y, int N, int H, int W, int C, int pad_t,
                                                         int pad_l, int OH, int OW) {
  constexpr int SPAN = TX + K - 1, ROWS = TY + K - 1;
  const int C4 = C >> 2, OWT = (OW + TX - 1) / TX, OHT = (OH + TY - 1) / TY;
  const int64_t total = (int64_t)N * OHT * OWT * C4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    int64_t t = e / C4;
    const int oxt = (int)(t % OWT); t /= OWT;
    const int oyt = (int)(t % OHT);
    const int n = (int)(t / OHT);
    const int c = c4 * 4, ox0 = oxt * TX, oy0 = oyt * TY, ix0 = ox0 - pad_l;
    float4 wk[K][K];
    dw_load_taps<K>(w, c, wk);
    float4 acc[TY][TX];
#pragma unroll
    for (int r = 0; r < TY; ++r)
#pragma unroll
      for (int q = 0; q < TX; ++q) acc[r][q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ri = 0; ri < ROWS; ++ri) {  // input row oy0 - pad_t + ri: tap row ky = ri - r of output row r
      const int iy = oy0 - pad_t + ri;
      if (iy < 0 || iy >= H) continue;
      const float* row = x + (((int64_t)n * H + iy) * W) * C + c;
      float4 v[SPAN];
#pragma unroll
      for (int j = 0; j < SPAN; ++j) {
        const int ix = ix0 + j;
        v[j] = (ix >= 0 && ix < W) ? *reinterpret_cast<const float4*>(row + (int64_t)ix * C)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int r = 0; r < TY; ++r) {
        const int ky = ri - r;
        if (ky < 0 || ky >= K) continue;
#pragma unroll
        for (int j = 0; j < SPAN; ++j)
#pragma unroll
          for (int q = 0; q < TX; ++q) {
            const int kx = j - q;
            if (kx >= 0 && kx < K) fma4(acc[r][q], v[j], wk[ky][kx]);
          }
      }
    }
#pragma unroll
    for (int r = 0; r < TY; ++r) {
      if (oy0 + r >= OH) break;
      float* out = y + (((int64_t)n * OH + oy0 + r) * OW) * C + c;
#pragma unroll
      for (int q = 0; q < TX; ++q)
        if (ox0 + q < OW) *reinterpret_cast<float4*>(out + (int64_t)(ox0 + q) * C) = acc[r][q];
    }
  }
}

// stride-1 input gradient, TY x TX blocks: dx[iy][ix] = sum dy[iy + pad_t - ky][ix + pad_l - kx]
// w[ky][kx]; dy row oy0 + pad_t - (K-1) + ri serves output row r with ky = r + K - 1 - ri
template <int K, int TX, int TY>
__global__ __launch_bounds__(256) void dwconv_dx_s1_blk(const float* __restrict__ dy, const float* __restrict__ w,
                                                        float* __restrict__ dx, int N, int H, int W, int C, int pad_t,
                                                        int pad_l, int OH, int OW) {
  constexpr int SPAN = TX + K - 1, ROWS = TY + K - 1;
  const int C4 = C >> 2, WT = (W + TX - 1) / TX, HT = (H + TY - 1) / TY;
  const int64_t total = (int64_t)N * HT * WT * C4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    int64_t t = e / C4;
    const int ixt = (int)(t % WT); t /= WT;
    const int iyt = (int)(t % HT);
    const int n = (int)(t / HT);
    const int c = c4 * 4, ix0 = ixt * TX, iy0 = iyt * TY;
    const int ox0 = ix0 + pad_l - (K - 1), oyb = iy0 + pad_t - (K - 1);
    float4 wk[K][K];
    dw_load_taps<K>(w, c, wk);
    float4 acc[TY][TX];
#pragma unroll
    for (int r = 0; r < TY; ++r)
#pragma unroll
      for (int q = 0; q < TX; ++q) acc[r][q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ri = 0; ri < ROWS; ++ri) {
      const int oy = oyb + ri;
      if (oy < 0 || oy >= OH) continue;
      const float* row = dy + (((int64_t)n * OH + oy) * OW) * C + c;
      float4 v[SPAN];
#pragma unroll
      for (int j = 0; j < SPAN; ++j) {
        const int ox = ox0 + j;
        v[j] = (ox >= 0 && ox < OW) ? *reinterpret_cast<const float4*>(row + (int64_t)ox * C)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int r = 0; r < TY; ++r) {
        const int ky = r + (K - 1) - ri;
        if (ky < 0 || ky >= K) continue;
#pragma unroll
        for (int j = 0; j < SPAN; ++j)
#pragma unroll
          for (int q = 0; q < TX; ++q) {
            const int kx = q + (K - 1) - j;
            if (kx >= 0 && kx < K) fma4(acc[r][q], v[j], wk[ky][kx]);
          }
      }
    }
#pragma unroll
    for (int r = 0; r < TY; ++r) {
      if (iy0 + r >= H) break;
      float* out = dx + (((int64_t)n * H + iy0 + r) * W) * C + c;
#pragma unroll
      for (int q = 0; q < TX; ++q)
        if (ix0 + q < W) *reinterpret_cast<float4*>(out + (int64_t)(ix0 + q) * C) = acc[r][q];
    }
  }
}

// stride-1 weight gradient, TY x TX output blocks per work item: the TY*TX dy quads and the
// TY + K - 1 input rows (SPAN quads each) are loaded once per item and update all K*K taps;
// block = 64 channel quads x 4 item lanes over a chunk of items, partials as in
// dwconv_dw_partial (part[chunk][c*KK + tap], a fixed-order column sum after)
template <int K, int TX, int TY>
__global__ __launch_bounds__(256) void dwconv_dw_partial_s1_blk(const float* __restrict__ dy,
                                                                const float* __restrict__ x, float* __restrict__ part,
                                                                int N, int H, int W, int C, int pad_t, int pad_l,
                                                                int OH, int OW, int64_t grp_per_chunk, int cl) {
  constexpr int KK = K * K, SPAN = TX + K - 1, ROWS = TY + K - 1;
  __shared__ float4 red[256];
  // cl channel-quad lanes x 256 / cl item lanes (cl = 64, or fewer for narrow maps: the
  // 24/48-channel stage-0 blocks would leave 58 of 64 lanes idle)
  const int lane = threadIdx.x % cl, ty = threadIdx.x / cl, nil = 256 / cl;
  const int C4 = C >> 2;
  const int c4 = blockIdx.x * cl + lane;
  const bool cok = c4 < C4;
  const int c = (cok ? c4 : 0) * 4;
  const int OWT = (OW + TX - 1) / TX, OHT = (OH + TY - 1) / TY;
  const int64_t ngrp = (int64_t)N * OHT * OWT;
  const int64_t g0 = (int64_t)blockIdx.y * grp_per_chunk;
  const int64_t g1 = min(ngrp, g0 + grp_per_chunk);
  float4 acc[K][K];
#pragma unroll
  for (int ky = 0; ky < K; ++ky)
#pragma unroll
    for (int kx = 0; kx < K; ++kx) acc[ky][kx] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (cok) {
    for (int64_t gi = g0 + ty; gi < g1; gi += nil) {
      const int oxt = (int)(gi % OWT);
      const int64_t t = gi / OWT;
      const int oyt = (int)(t % OHT);
      const int n = (int)(t / OHT);
      const int ox0 = oxt * TX, oy0 = oyt * TY;
      float4 g[TY][TX];
#pragma unroll
      for (int r = 0; r < TY; ++r)
#pragma unroll
        for (int q = 0; q < TX; ++q)
          g[r][q] = (oy0 + r < OH && ox0 + q < OW)
                        ? *reinterpret_cast<const float4*>(dy + (((int64_t)n * OH + oy0 + r) * OW + ox0 + q) * C + c)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int ri = 0; ri < ROWS; ++ri) {
        const int iy = oy0 - pad_t + ri;
        if (iy < 0 || iy >= H) continue;
        const float* row = x + (((int64_t)n * H + iy) * W) * C + c;
        float4 v[SPAN];
#pragma unroll
        for (int j = 0; j < SPAN; ++j) {
          const int ix = ox0 - pad_l + j;
          v[j] = (ix >= 0 && ix < W) ? *reinterpret_cast<const float4*>(row + (int64_t)ix * C)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int r = 0; r < TY; ++r) {
          const int ky = ri - r;
          if (ky < 0 || ky >= K) continue;
#pragma unroll
          for (int j = 0; j < SPAN; ++j)
#pragma unroll
            for (int q = 0; q < TX; ++q) {
              const int kx = j - q;
              if (kx >= 0 && kx < K) fma4(acc[ky][kx], g[r][q], v[j]);
            }
        }
      }
    }
  }
  float* dst = part + (int64_t)blockIdx.y * C * KK;
#pragma unroll
  for (int k = 0; k < KK; ++k) {
    red[threadIdx.x] = acc[k / K][k % K];
    __syncthreads();
    if (ty == 0 && cok) {
      float4 sum = red[lane];
      for (int q = 1; q < nil; ++q) {  // item lanes in order
        const float4 v = red[q * cl + lane];
        sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
      }
      dst[(int64_t)(c + 0) * KK + k] = sum.x;
      dst[(int64_t)(c + 1) * KK + k] = sum.y;
      dst[(int64_t)(c + 2) * KK + k] = sum.z;
      dst[(int64_t)(c + 3) * KK + k] = sum.w;
    }
    __syncthreads();
  }
}

// tile rows per thread of the stride-1 block kernels (MDEMI_DW_TY: A/B; 1 = the one-row kernels)
static int dw_ty() {
  static int ty = [] {
    const char* v = getenv("MDEMI_DW_TY");
    const int t = v ? atoi(v) : 4;
    return (t == 1 || t == 2 || t == 4) ? t : 4;
  }();
  return ty;
}

static int dw_chunks(int C, int64_t npix) {
  const int gx = (int)cdiv(C / 4, 64);
  int64_t ch = cdiv(1024, gx);
  const int64_t maxch = cdiv(npix, 64);
  if (ch > maxch) ch = maxch;
  if (ch < 1) ch = 1;
  return (int)ch;
}

// ---------------------------------------------------------------------------
// spatial reductions: out[n][c] = scale * sum_p a*b   (chunked partials + fixed-order final sum)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void spatial_partial(const float* __restrict__ a, const float* __restrict__ b,
                                                       float* __restrict__ part, int64_t HW, int C, int nchunk,
                                                       int64_t per_chunk) {
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int C4 = C >> 2;
  const int c4 = blockIdx.x * 64 + lane;
  const int n = blockIdx.z, ch = blockIdx.y;
  const bool cok = c4 < C4;
  const int64_t p0 = (int64_t)ch * per_chunk, p1 = min(HW, p0 + per_chunk);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (cok) {
    const int64_t base = (int64_t)n * HW * C + (int64_t)c4 * 4;
#pragma unroll 4
    for (int64_t p = p0 + ty; p < p1; p += 4) {  // unrolled: loads in flight, sums in row order
      const float4 u = *reinterpret_cast<const float4*>(a + base + p * C);
      if (b) {
        const float4 v = *reinterpret_cast<const float4*>(b + base + p * C);
        s.x = fmaf(u.x, v.x, s.x); s.y = fmaf(u.y, v.y, s.y); s.z = fmaf(u.z, v.z, s.z); s.w = fmaf(u.w, v.w, s.w);
      } else {
        s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
      }
    }
  }
  red[ty][lane] = s;
  __syncthreads();
  if (ty == 0 && cok) {
    float4 t = red[0][lane];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const float4 v = red[q][lane];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    *reinterpret_cast<float4*>(part + ((int64_t)n * nchunk + ch) * C + c4 * 4) = t;
  }
}

__global__ __launch_bounds__(256) void spatial_final(const float* __restrict__ part, float* __restrict__ out, int N,
                                                     int C, int nchunk, float scale) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)N * C) return;
  const int n = (int)(e / C), c = (int)(e % C);
  double s = 0.0;  // fixed-order fp64 combine of the chunk partials (unrolled: loads in flight)
#pragma unroll 8
  for (int k = 0; k < nchunk; ++k) s += (double)part[((int64_t)n * nchunk + k) * C + c];
  out[e] = (float)(s * (double)scale);
}

static int spatial_chunks(int N, int64_t HW, int C) {
  const int gx = (int)cdiv(C / 4, 64);
  int64_t ch = cdiv(2048, (int64_t)gx * N);
  const int64_t maxch = cdiv(HW, 64);
  if (ch > maxch) ch = maxch;
  if (ch > 4096) ch = 4096;
  return (int)(ch < 1 ? 1 : ch);
}

__global__ __launch_bounds__(256) void chan_scale_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                         const float* __restrict__ add, float* __restrict__ y,
                                                         int64_t HW, int C, int64_t total4,
                                                         __bf16* __restrict__ y16 = nullptr) {
  const int C4 = C >> 2;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total4; e += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    const int64_t n = e / ((int64_t)HW * C4);
    const float4 v = reinterpret_cast<const float4*>(x)[e];
    const float4 s = *reinterpret_cast<const float4*>(g + n * C + c4 * 4);
    float4 o = make_float4(v.x * s.x, v.y * s.y, v.z * s.z, v.w * s.w);
    if (add) {
      const float4 a = *reinterpret_cast<const float4*>(add + n * C + c4 * 4);
      o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
    }
    reinterpret_cast<float4*>(y)[e] = o;
    if (y16) {  // the RNE bf16 copy a following bf16 GEMM (conv_pwl) reads
      typedef __bf16 b4 __attribute__((ext_vector_type(4)));
      typedef float f4v __attribute__((ext_vector_type(4)));
      const f4v ov = {o.x, o.y, o.z, o.w};
      reinterpret_cast<b4*>(y16)[e] = __builtin_convertvector(ov, b4);
    }
  }
}

// ---------------------------------------------------------------------------
// SqueezeExcite gate MLP, split so that every stage has N x (R/4 or C/256)
// workgroups (one workgroup per image left 240 of 256 CUs idle at batch 16):
//   hid[n][r]  = br[r] + sum_c wr[r][c] pooled[n][c]        (wave per (n, r))
//   gate[n][c] = sigmoid(be[c] + sum_r we[c][r] silu(hid[n][r]))   (thread per (n, c))
// ---------------------------------------------------------------------------
constexpr int SE_MAXC = 4096, SE_MAXR = 256;

__global__ __launch_bounds__(256) void se_hid_kernel(const float* __restrict__ pooled, const float* __restrict__ wr,
                                                     const float* __restrict__ br, float* __restrict__ hid, int C,
                                                     int R) {
  const int n = blockIdx.x, lane = threadIdx.x & 63;
  const int r = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* wrow = wr + (int64_t)r * C;
  const float* pv = pooled + (int64_t)n * C;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s = fmaf(wrow[c], pv[c], s);
  s = wave_sum(s);
  if (lane == 0) hid[(int64_t)n * R + r] = s + br[r];
}

__global__ __launch_bounds__(256) void se_gate_kernel(const float* __restrict__ hid, const float* __restrict__ we,
                                                      const float* __restrict__ be, float* __restrict__ gate, int C,
                                                      int R) {
  __shared__ float sh[SE_MAXR];
  const int n = blockIdx.x;
  for (int r = threadIdx.x; r < R; r += 256) sh[r] = silu_f(hid[(int64_t)n * R + r]);
  __syncthreads();
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  const float* wrow = we + (int64_t)c * R;
  float s = be[c];
  for (int r = 0; r < R; ++r) s = fmaf(wrow[r], sh[r], s);
  gate[(int64_t)n * C + c] = sigmoid_f(s);
}

// backward, per image: de = dgate * g(1-g); dz = (we^T de) * silu'(hid); dpooled = wr^T dz
__global__ __launch_bounds__(256) void se_dz_kernel(const float* __restrict__ we, const float* __restrict__ hid,
                                                    const float* __restrict__ gate, const float* __restrict__ dgate,
                                                    float* __restrict__ de_out, float* __restrict__ dz_out, int C,
                                                    int R) {
  const int n = blockIdx.x, lane = threadIdx.x & 63;
  const int r = blockIdx.y * 4 + (threadIdx.x >> 6);
  const float* gv = gate + (int64_t)n * C;
  const float* dgv = dgate + (int64_t)n * C;
  if (blockIdx.y == 0)  // de is also the conv_expand bias/weight gradient's input
    for (int c = threadIdx.x; c < C; c += 256) de_out[(int64_t)n * C + c] = dgv[c] * gv[c] * (1.f - gv[c]);
  if (r >= R) return;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float g = gv[c];
    s = fmaf(we[(int64_t)c * R + r], dgv[c] * g * (1.f - g), s);
  }
  s = wave_sum(s);
  if (lane == 0) dz_out[(int64_t)n * R + r] = s * silu_grad_f(hid[(int64_t)n * R + r]);
}

__global__ __launch_bounds__(256) void se_dpooled_kernel(const float* __restrict__ wr, const float* __restrict__ dz,
                                                         float* __restrict__ dpooled, int C, int R, float scale) {
  __shared__ float sdz[SE_MAXR];
  const int n = blockIdx.x;
  for (int r = threadIdx.x; r < R; r += 256) sdz[r] = dz[(int64_t)n * R + r];
  __syncthreads();
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s = fmaf(wr[(int64_t)r * C + c], sdz[r], s);
  dpooled[(int64_t)n * C + c] = s * scale;  // scale 1 / HW: the per-position gradient of the mean
}

// parameter gradients, summed over the N images in order
__global__ __launch_bounds__(256) void se_gate_wgrad_kernel(const float* __restrict__ pooled,
                                                            const float* __restrict__ hid,
                                                            const float* __restrict__ de, const float* __restrict__ dz,
                                                            float* __restrict__ dwr, float* __restrict__ dbr,
                                                            float* __restrict__ dwe, float* __restrict__ dbe, int N,
                                                            int C, int R) {
  const int64_t RC = (int64_t)R * C;
  const int64_t total = 2 * RC + C + R;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    double s = 0.0;  // sums over the N images in fp64 (N is small; these are tiny tensors)
    if (e < RC) {  // dwr[r][c] = sum_n dz[n][r] * pooled[n][c]
      const int r = (int)(e / C), c = (int)(e % C);
      for (int n = 0; n < N; ++n) s += (double)dz[(int64_t)n * R + r] * pooled[(int64_t)n * C + c];
      dwr[e] = (float)s;
    } else if (e < 2 * RC) {  // dwe[c][r] = sum_n de[n][c] * silu(hid[n][r])
      const int64_t f = e - RC;
      const int c = (int)(f / R), r = (int)(f % R);
      for (int n = 0; n < N; ++n) s += (double)de[(int64_t)n * C + c] * silu_f(hid[(int64_t)n * R + r]);
      dwe[f] = (float)s;
    } else if (e < 2 * RC + C) {
      const int c = (int)(e - 2 * RC);
      for (int n = 0; n < N; ++n) s += de[(int64_t)n * C + c];
      dbe[c] = (float)s;
    } else {
      const int r = (int)(e - 2 * RC - C);
      for (int n = 0; n < N; ++n) s += dz[(int64_t)n * R + r];
      dbr[r] = (float)s;
    }
  }
}

__global__ __launch_bounds__(256) void nchw_to_nhwc_pad_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               int N, int C, int64_t HW, int Cp) {
  const int64_t total = (int64_t)N * HW;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t n = e / HW, p = e % HW;
    float* dst = y + e * Cp;
    for (int c = 0; c < Cp; ++c) dst[c] = c < C ? x[(n * C + c) * HW + p] : 0.f;
  }
}

template <int K, int S>
static void launch_dw_fwd(const float* x, const float* w, float* y, int N, int H, int W, int C, int pt, int pl, int OH,
                          int OW, hipStream_t st) {
  if (S == 1 && dw_ty() > 1) {
    constexpr int TX = 4;
    const int TY = dw_ty();
    const int64_t total = (int64_t)N * ((OH + TY - 1) / TY) * ((OW + TX - 1) / TX) * (C / 4);
    if (TY == 2)
      hipLaunchKernelGGL((dwconv_fwd_s1_blk<K, TX, 2>), dim3(grid_1d(total)), dim3(256), 0, st, x, w, y, N, H, W, C,
                         pt, pl, OH, OW);
    else
      hipLaunchKernelGGL((dwconv_fwd_s1_blk<K, TX, 4>), dim3(grid_1d(total)), dim3(256), 0, st, x, w, y, N, H, W, C,
                         pt, pl, OH, OW);
    return;
  }
  constexpr int TX = S == 1 ? 4 : 2;
  const int64_t total = (int64_t)N * OH * ((OW + TX - 1) / TX) * (C / 4);
  hipLaunchKernelGGL((dwconv_fwd_kernel<K, S, TX>), dim3(grid_1d(total)), dim3(256), 0, st, x, w, y, N, H, W, C, pt,
                     pl, OH, OW);
}
template <int K, int S>
static void launch_dw_bwd(const float* dy, const float* x, const float* w, float* dx, float* part, int N, int H,
                          int W, int C, int pt, int pl, int OH, int OW, hipStream_t st) {
  if (dx && S == 1 && dw_ty() > 1) {
    constexpr int TX = 4;
    const int TY = dw_ty();
    const int64_t total = (int64_t)N * ((H + TY - 1) / TY) * ((W + TX - 1) / TX) * (C / 4);
    if (TY == 2)
      hipLaunchKernelGGL((dwconv_dx_s1_blk<K, TX, 2>), dim3(grid_1d(total)), dim3(256), 0, st, dy, w, dx, N, H, W, C,
                         pt, pl, OH, OW);
    else
      hipLaunchKernelGGL((dwconv_dx_s1_blk<K, TX, 4>), dim3(grid_1d(total)), dim3(256), 0, st, dy, w, dx, N, H, W, C,
                         pt, pl, OH, OW);
  } else if (dx) {
    constexpr int TX = 4;
    const int64_t total = (int64_t)N * H * ((W + TX - 1) / TX) * (C / 4);
    if (S == 1)
      hipLaunchKernelGGL((dwconv_dx_s1_kernel<K, TX>), dim3(grid_1d(total)), dim3(256), 0, st, dy, w, dx, N, H, W, C,
                         pt, pl, OH, OW);
    else
      hipLaunchKernelGGL((dwconv_dx_kernel<K, S, TX>), dim3(grid_1d(total)), dim3(256), 0, st, dy, w, dx, N, H, W,
                         C, pt, pl, OH, OW);
  }
  if (part && S == 1 && dw_ty() > 1) {
    constexpr int TXW = 4;
    const int TY = dw_ty();
    const int64_t npix = (int64_t)N * OH * OW;
    const int ch = dw_chunks(C, npix);
    const int64_t ngrp = (int64_t)N * ((OH + TY - 1) / TY) * ((OW + TXW - 1) / TXW);
    int cl = 8;
    while (cl < 64 && cl < C / 4) cl *= 2;
    dim3 grid((unsigned)cdiv(C / 4, cl), (unsigned)ch);
    if (TY == 2)
      hipLaunchKernelGGL((dwconv_dw_partial_s1_blk<K, TXW, 2>), grid, dim3(256), 0, st, dy, x, part, N, H, W, C, pt,
                         pl, OH, OW, cdiv(ngrp, ch), cl);
    else
      hipLaunchKernelGGL((dwconv_dw_partial_s1_blk<K, TXW, 4>), grid, dim3(256), 0, st, dy, x, part, N, H, W, C, pt,
                         pl, OH, OW, cdiv(ngrp, ch), cl);
  } else if (part && S == 1) {
    constexpr int TXW = 4;
    const int64_t npix = (int64_t)N * OH * OW;
    const int ch = dw_chunks(C, npix);
    const int64_t ngrp = (int64_t)N * OH * ((OW + TXW - 1) / TXW);
    dim3 grid((unsigned)cdiv(C / 4, 64), (unsigned)ch);
    hipLaunchKernelGGL((dwconv_dw_partial_s1<K, TXW>), grid, dim3(256), 0, st, dy, x, part, N, H, W, C, pt, pl, OH,
                       OW, cdiv(ngrp, ch));
  } else if (part) {
    const int64_t npix = (int64_t)N * OH * OW;
    const int ch = dw_chunks(C, npix);
    dim3 grid((unsigned)cdiv(C / 4, 64), (unsigned)ch);
    hipLaunchKernelGGL((dwconv_dw_partial<K, S>), grid, dim3(256), 0, st, dy, x, part, N, H, W, C, pt, pl, OH, OW,
                       cdiv(npix, ch));
  }
}

}  // namespace mdemi

using namespace mdemi;

#define MDEMI_DW_DISPATCH(FN, ...)                                          \
  do {                                                                      \
    if (K == 3 && stride == 1) FN<3, 1>(__VA_ARGS__);                       \
    else if (K == 3 && stride == 2) FN<3, 2>(__VA_ARGS__);                  \
    else if (K == 5 && stride == 1) FN<5, 1>(__VA_ARGS__);                  \
    else if (K == 5 && stride == 2) FN<5, 2>(__VA_ARGS__);                  \
    else {                                                                  \
      set_error("dwconv: unsupported kernel %d / stride %d", K, stride);    \
      return MDEMI_EUNSUP;                                                  \
    }                                                                       \
  } while (0)

extern "C" int mdemi_dwconv_fwd(const float* x, const float* w, float* y, int32_t N, int32_t H, int32_t W, int32_t C,
                                int32_t K, int32_t stride, int32_t pad_t, int32_t pad_l, int32_t OH, int32_t OW,
                                void* stream) {
  MDEMI_REQUIRE(x && w && y && N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0, "dwconv_fwd: bad args");
  MDEMI_REQUIRE(C % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0,
                "dwconv_fwd: needs C %% 4 == 0 and 16-B aligned activations (C=%d)", C);
  MDEMI_REQUIRE(pad_t >= 0 && pad_l >= 0 && pad_t < K && pad_l < K, "dwconv_fwd: bad padding");
  hipStream_t st = (hipStream_t)stream;
  MDEMI_DW_DISPATCH(launch_dw_fwd, x, w, y, N, H, W, C, pad_t, pad_l, OH, OW, st);
  return check_launch("dwconv_fwd");
}

extern "C" size_t mdemi_dwconv_bwd_workspace_size(int32_t N, int32_t C, int32_t K, int32_t OH, int32_t OW) {
  const int64_t npix = (int64_t)N * OH * OW;
  const int ch = dw_chunks(C, npix);
  return align_up((size_t)ch * C * K * K * sizeof(float), 256) + colsum_ws_bytes(ch, (int64_t)C * K * K);
}

extern "C" int mdemi_dwconv_bwd(const float* dy, const float* x, const float* w, float* dx, float* dw, int32_t N,
                                int32_t H, int32_t W, int32_t C, int32_t K, int32_t stride, int32_t pad_t,
                                int32_t pad_l, int32_t OH, int32_t OW, void* workspace, void* stream) {
  MDEMI_REQUIRE(dy && x && w && N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0, "dwconv_bwd: bad args");
  MDEMI_REQUIRE(C % 4 == 0, "dwconv_bwd: needs C %% 4 == 0");
  MDEMI_REQUIRE(pad_t >= 0 && pad_l >= 0 && pad_t < K && pad_l < K, "dwconv_bwd: bad padding");
  if (dw && !workspace) { set_error("dwconv_bwd: workspace required"); return MDEMI_EWORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  float* part = dw ? (float*)workspace : nullptr;
  MDEMI_DW_DISPATCH(launch_dw_bwd, dy, x, w, dx, part, N, H, W, C, pad_t, pad_l, OH, OW, st);
  if (dw) {
    const int64_t npix = (int64_t)N * OH * OW;
    const int ch = dw_chunks(C, npix);
    const int64_t cols = (int64_t)C * K * K;
    char* cws = (char*)workspace + align_up((size_t)ch * cols * sizeof(float), 256);
    int rc = colsum_launch(part, ch, cols, cols, dw, 0, cws, st);
    if (rc) return rc;
  }
  return check_launch("dwconv_bwd");
}

extern "C" size_t mdemi_spatial_reduce_workspace_size(int32_t N, int64_t HW, int32_t C) {
  return align_up((size_t)N * spatial_chunks(N, HW, C) * C * sizeof(float), 256);
}

extern "C" int mdemi_spatial_reduce(const float* a, const float* b, float* out, int32_t N, int64_t HW, int32_t C,
                                    float scale, void* workspace, void* stream) {
  MDEMI_REQUIRE(a && out && N > 0 && HW > 0 && C > 0 && C % 4 == 0, "spatial_reduce: bad args (C %% 4 == 0)");
  if (!workspace) { set_error("spatial_reduce: workspace required"); return MDEMI_EWORKSPACE; }
  const int ch = spatial_chunks(N, HW, C);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)cdiv(C / 4, 64), (unsigned)ch, (unsigned)N);
  hipLaunchKernelGGL(spatial_partial, grid, dim3(256), 0, st, a, b, (float*)workspace, HW, C, ch, cdiv(HW, ch));
  hipLaunchKernelGGL(spatial_final, dim3(grid_1d((int64_t)N * C)), dim3(256), 0, st, (const float*)workspace, out, N,
                     C, ch, scale);
  return check_launch("spatial_reduce");
}

extern "C" int mdemi_chan_scale(const float* x, const float* g, const float* add, float* y, int32_t N, int64_t HW,
                                int32_t C, void* stream) {
  return mdemi_chan_scale16(x, g, add, y, nullptr, N, HW, C, stream);
}

extern "C" int mdemi_chan_scale16(const float* x, const float* g, const float* add, float* y, void* y16, int32_t N,
                                  int64_t HW, int32_t C, void* stream) {
  MDEMI_REQUIRE(x && g && y && N > 0 && HW > 0 && C > 0 && C % 4 == 0, "chan_scale: bad args (C %% 4 == 0)");
  MDEMI_REQUIRE(!y16 || ((uintptr_t)y16 & 7) == 0, "chan_scale16: y16 must be 8-B aligned");
  const int64_t total4 = (int64_t)N * HW * C / 4;
  hipLaunchKernelGGL(chan_scale_kernel, dim3(grid_1d(total4)), dim3(256), 0, (hipStream_t)stream, x, g, add, y, HW, C,
                     total4, (__bf16*)y16);
  return check_launch("chan_scale");
}

extern "C" int mdemi_se_gate_fwd(const float* pooled, const float* wr, const float* br, const float* we,
                                 const float* be, float* hid, float* gate, int32_t N, int32_t C, int32_t R,
                                 void* stream) {
  MDEMI_REQUIRE(pooled && wr && br && we && be && hid && gate && N > 0 && C > 0 && R > 0, "se_gate_fwd: bad args");
  MDEMI_REQUIRE(C <= SE_MAXC && R <= SE_MAXR, "se_gate_fwd: C=%d R=%d exceed %d/%d", C, R, SE_MAXC, SE_MAXR);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(se_hid_kernel, dim3(N, (unsigned)cdiv(R, 4)), dim3(256), 0, st, pooled, wr, br, hid, C, R);
  hipLaunchKernelGGL(se_gate_kernel, dim3(N, (unsigned)cdiv(C, 256)), dim3(256), 0, st, hid, we, be, gate, C, R);
  return check_launch("se_gate_fwd");
}

extern "C" size_t mdemi_se_gate_bwd_workspace_size(int32_t N, int32_t C, int32_t R) {
  return align_up((size_t)N * (C + R) * sizeof(float), 256);
}

extern "C" int mdemi_se_gate_bwd(const float* pooled, const float* wr, const float* we, const float* hid,
                                 const float* gate, const float* dgate, float* dpooled, float* dwr, float* dbr,
                                 float* dwe, float* dbe, int32_t N, int32_t C, int32_t R, float dpooled_scale,
                                 void* workspace, void* stream) {
  MDEMI_REQUIRE(pooled && wr && we && hid && gate && dgate && dpooled && dwr && dbr && dwe && dbe && N > 0 && C > 0 &&
                    R > 0, "se_gate_bwd: bad args");
  MDEMI_REQUIRE(C <= SE_MAXC && R <= SE_MAXR, "se_gate_bwd: C=%d R=%d exceed %d/%d", C, R, SE_MAXC, SE_MAXR);
  if (!workspace) { set_error("se_gate_bwd: workspace required"); return MDEMI_EWORKSPACE; }
  float* de = (float*)workspace;
  float* dz = de + (int64_t)N * C;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(se_dz_kernel, dim3(N, (unsigned)cdiv(R, 4)), dim3(256), 0, st, we, hid, gate, dgate, de, dz, C, R);
  hipLaunchKernelGGL(se_dpooled_kernel, dim3(N, (unsigned)cdiv(C, 256)), dim3(256), 0, st, wr, dz, dpooled, C, R,
                     dpooled_scale);
  const int64_t total = 2 * (int64_t)R * C + C + R;
  hipLaunchKernelGGL(se_gate_wgrad_kernel, dim3(grid_1d(total)), dim3(256), 0, st, pooled, hid, de, dz, dwr, dbr, dwe,
                     dbe, N, C, R);
  return check_launch("se_gate_bwd");
}

extern "C" int mdemi_nchw_to_nhwc_pad(const float* x, float* y, int32_t N, int32_t C, int64_t HW, int32_t Cp,
                                      void* stream) {
  MDEMI_REQUIRE(x && y && N > 0 && C > 0 && HW > 0 && Cp >= C, "nchw_to_nhwc_pad: bad args");
  hipLaunchKernelGGL(nchw_to_nhwc_pad_kernel, dim3(grid_1d((int64_t)N * HW)), dim3(256), 0, (hipStream_t)stream, x, y,
                     N, C, HW, Cp);
  return check_launch("nchw_to_nhwc_pad");
}
