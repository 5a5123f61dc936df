// KxK convolution to ONE output channel over an NHWC map (DispHead.conv1,
// NewCRFDepth.py:155: Conv2d(128, 1, 3, padding=1)).  A GEMM with N = 1 would
// waste 127/128 of every MFMA tile, so this is a memory-bound sweep instead:
//   fwd   one wave per output pixel, lanes across channels (float4), taps in
//         registers, wave reduction;   y = b + sum_{tap,c} x * w
//   dgrad thread per (input pixel, channel quad): 9 scalar dy taps
//   wgrad per-block partials of dy * x over pixels, deterministic reduce.
// Weights are read in the reference layout [1][C][KH][KW].
#include "common.h"

namespace mdemi {

constexpr int HC_THREADS = 256;

struct HcGeom {
  int N, H, W, C, K, pad;
};

__global__ __launch_bounds__(HC_THREADS) void headconv_fwd_kernel(const float* __restrict__ x,
                                                                   const float* __restrict__ w,
                                                                   const float* __restrict__ b, float* __restrict__ y,
                                                                   HcGeom g) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * HC_THREADS + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * HC_THREADS) >> 6;
  const int64_t npix = (int64_t)g.N * g.H * g.W;
  const int C4 = g.C / 4;
  const int KK = g.K * g.K;
  const float bias = b ? b[0] : 0.f;
  for (int64_t p = wave; p < npix; p += nwaves) {
    const int xx = (int)(p % g.W);
    const int64_t t = p / g.W;
    const int yy = (int)(t % g.H);
    const int n = (int)(t / g.H);
    float acc = 0.f;
    for (int tap = 0; tap < KK; ++tap) {
      const int iy = yy + tap / g.K - g.pad, ix = xx + tap % g.K - g.pad;
      if (iy < 0 || iy >= g.H || ix < 0 || ix >= g.W) continue;  // wave-uniform
      const float4* src = reinterpret_cast<const float4*>(x + (((int64_t)n * g.H + iy) * g.W + ix) * g.C);
      for (int c4 = lane; c4 < C4; c4 += 64) {
        const float4 v = src[c4];
        const int c = 4 * c4;
        acc = fmaf(v.x, w[(c + 0) * KK + tap], acc);
        acc = fmaf(v.y, w[(c + 1) * KK + tap], acc);
        acc = fmaf(v.z, w[(c + 2) * KK + tap], acc);
        acc = fmaf(v.w, w[(c + 3) * KK + tap], acc);
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) y[p] = acc + bias;
  }
}

// dx[n,y,x,c] = sum_tap dy[n, y - ky + pad, x - kx + pad] * w[c][ky][kx]
__global__ __launch_bounds__(HC_THREADS) void headconv_dgrad_kernel(const float* __restrict__ dy,
                                                                    const float* __restrict__ w,
                                                                    float* __restrict__ dx, HcGeom g) {
  const int C4 = g.C / 4;
  const int KK = g.K * g.K;
  const int64_t total = (int64_t)g.N * g.H * g.W * C4;
  for (int64_t e = (int64_t)blockIdx.x * HC_THREADS + threadIdx.x; e < total; e += (int64_t)gridDim.x * HC_THREADS) {
    const int c4 = (int)(e % C4);
    const int64_t p = e / C4;
    const int xx = (int)(p % g.W);
    const int64_t t = p / g.W;
    const int yy = (int)(t % g.H);
    const int n = (int)(t / g.H);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int c = 4 * c4;
    for (int tap = 0; tap < KK; ++tap) {
      const int oy = yy - tap / g.K + g.pad, ox = xx - tap % g.K + g.pad;
      if (oy < 0 || oy >= g.H || ox < 0 || ox >= g.W) continue;
      const float d = dy[((int64_t)n * g.H + oy) * g.W + ox];
      acc.x = fmaf(d, w[(c + 0) * KK + tap], acc.x);
      acc.y = fmaf(d, w[(c + 1) * KK + tap], acc.y);
      acc.z = fmaf(d, w[(c + 2) * KK + tap], acc.z);
      acc.w = fmaf(d, w[(c + 3) * KK + tap], acc.w);
    }
    reinterpret_cast<float4*>(dx)[e] = acc;
  }
}

// partial[blk][tap*C + c] (+ partial[blk][C*KK] = sum dy for the bias); channel-fastest
// so a wave's loads of x are contiguous
__global__ __launch_bounds__(HC_THREADS) void headconv_wgrad_partial(const float* __restrict__ dy,
                                                                     const float* __restrict__ x,
                                                                     float* __restrict__ part, HcGeom g,
                                                                     int64_t pix_per_blk) {
  const int KK = g.K * g.K;
  const int nout = g.C * KK;
  const int64_t npix = (int64_t)g.N * g.H * g.W;
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_blk;
  const int64_t p1 = min(npix, p0 + pix_per_blk);
  float* P = part + (int64_t)blockIdx.x * (nout + 1);
  for (int o = threadIdx.x; o <= nout; o += HC_THREADS) {
    float s = 0.f;
    if (o == nout) {
      for (int64_t p = p0; p < p1; ++p) s += dy[p];
    } else {
      const int tap = o / g.C, c = o % g.C;
      const int ky = tap / g.K, kx = tap % g.K;
      for (int64_t p = p0; p < p1; ++p) {
        const int xx = (int)(p % g.W);
        const int64_t t = p / g.W;
        const int yy = (int)(t % g.H);
        const int n = (int)(t / g.H);
        const int iy = yy + ky - g.pad, ix = xx + kx - g.pad;
        if (iy < 0 || iy >= g.H || ix < 0 || ix >= g.W) continue;
        s = fmaf(dy[p], x[(((int64_t)n * g.H + iy) * g.W + ix) * g.C + c], s);
      }
    }
    P[o] = s;
  }
}

__global__ void headconv_wgrad_reduce(const float* __restrict__ part, int nblk, int nout, int C, int KK,
                                      float* __restrict__ dw, float* __restrict__ db) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o > nout) return;
  float s = 0.f;
  for (int i = 0; i < nblk; ++i) s += part[(int64_t)i * (nout + 1) + o];
  if (o < nout) dw[(o % C) * KK + o / C] = s;  // reference layout [1][C][KH][KW]
  else if (db) db[0] = s;
}

static int hc_grid(int64_t work, int per) {
  const int64_t nb = cdiv(work, per);
  return (int)(nb < 8192 ? (nb < 1 ? 1 : nb) : 8192);
}
static int64_t hc_pix_per_blk(int64_t npix) { return cdiv(npix, 512); }

}  // namespace mdemi

using namespace mdemi;

static int hc_check(int32_t N, int32_t H, int32_t W, int32_t C, int32_t K, int32_t pad) {
  MDEMI_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0 && K > 0 && pad >= 0 && 2 * pad == K - 1,
                "headconv: needs C %% 4 == 0 and 'same' padding (C=%d K=%d pad=%d)", C, K, pad);
  return MDEMI_OK;
}

extern "C" int mdemi_headconv_fwd(const float* x, const float* w, const float* b, float* y, int32_t N, int32_t H,
                                  int32_t W, int32_t C, int32_t K, int32_t pad, void* stream) {
  MDEMI_REQUIRE(x && w && y, "headconv_fwd: null pointer");
  int rc = hc_check(N, H, W, C, K, pad);
  if (rc) return rc;
  HcGeom g{N, H, W, C, K, pad};
  const int64_t npix = (int64_t)N * H * W;
  hipLaunchKernelGGL(headconv_fwd_kernel, dim3(hc_grid(npix, HC_THREADS / 64)), dim3(HC_THREADS), 0,
                     (hipStream_t)stream, x, w, b, y, g);
  return check_launch("headconv_fwd");
}

extern "C" size_t mdemi_headconv_wgrad_workspace_size(int32_t N, int32_t H, int32_t W, int32_t C, int32_t K) {
  const int64_t npix = (int64_t)N * H * W;
  const int64_t nblk = cdiv(npix, hc_pix_per_blk(npix));
  return (size_t)nblk * ((size_t)C * K * K + 1) * sizeof(float);
}

extern "C" int mdemi_headconv_bwd(const float* dy, const float* x, const float* w, float* dx, float* dw, float* db,
                                  int32_t N, int32_t H, int32_t W, int32_t C, int32_t K, int32_t pad,
                                  void* workspace, void* stream) {
  MDEMI_REQUIRE(dy && x && w, "headconv_bwd: null pointer");
  int rc = hc_check(N, H, W, C, K, pad);
  if (rc) return rc;
  HcGeom g{N, H, W, C, K, pad};
  hipStream_t st = (hipStream_t)stream;
  const int64_t npix = (int64_t)N * H * W;
  if (dx)
    hipLaunchKernelGGL(headconv_dgrad_kernel, dim3(hc_grid(npix * C / 4, HC_THREADS)), dim3(HC_THREADS), 0, st, dy, w,
                       dx, g);
  if (dw) {
    if (!workspace) { set_error("headconv_bwd: workspace required"); return MDEMI_EWORKSPACE; }
    const int64_t ppb = hc_pix_per_blk(npix);
    const int nblk = (int)cdiv(npix, ppb);
    const int nout = C * K * K;
    hipLaunchKernelGGL(headconv_wgrad_partial, dim3(nblk), dim3(HC_THREADS), 0, st, dy, x, (float*)workspace, g, ppb);
    hipLaunchKernelGGL(headconv_wgrad_reduce, dim3((nout + 256) / 256), dim3(256), 0, st, (const float*)workspace, nblk,
                       nout, C, K * K, dw, db);
  }
  return check_launch("headconv_bwd");
}
