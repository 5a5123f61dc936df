// KxK convolution to ONE output channel over an NHWC map (DispHead.conv1,
// NewCRFDepth.py:155: Conv2d(128, 1, 3, padding=1)).  A GEMM with N = 1 would
// waste 127/128 of every MFMA tile, so this is a memory-bound sweep instead:
//   fwd   32 lanes per output pixel across channel quads, weights transposed
//         to [tap][C] in LDS, 32-lane reduction;   y = b + sum_{tap,c} x * w
//   dgrad thread per (input pixel, channel quad): 9 scalar dy taps x LDS weights
//   wgrad per-block partials of dy * x (9 tap accumulators per channel quad in
//         registers, 8 pixel rows folded in LDS), deterministic reduce.
// Weights are read in the reference layout [1][C][KH][KW].
#include "common.h"

namespace mdemi {

constexpr int HC_THREADS = 256;
constexpr int HC_MAXC = 512;  // channels staged in LDS (weights transposed to [tap][C])

struct HcGeom {
  int N, H, W, C, K, pad;
};

// w [1][C][K][K] -> LDS wT[tap][C]
__device__ __forceinline__ void stage_wT(float* wT, const float* __restrict__ w, const HcGeom& g) {
  const int KK = g.K * g.K;
  for (int e = threadIdx.x; e < g.C * KK; e += HC_THREADS) wT[(e % KK) * g.C + e / KK] = w[e];
}

// y[p] = b + sum_{tap,c} x[p + tap] * w[c][tap]; 32 lanes per pixel (float4 channels), 8 pixels per block pass
__global__ __launch_bounds__(HC_THREADS) void headconv_fwd_kernel(const float* __restrict__ x,
                                                                   const float* __restrict__ w,
                                                                   const float* __restrict__ b, float* __restrict__ y,
                                                                   HcGeom g) {
  __shared__ __attribute__((aligned(16))) float wT[9 * HC_MAXC];
  stage_wT(wT, w, g);
  __syncthreads();
  const int sub = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int64_t npix = (int64_t)g.N * g.H * g.W;
  const int C4 = g.C / 4, KK = g.K * g.K;
  const float bias = b ? b[0] : 0.f;
  for (int64_t p = (int64_t)blockIdx.x * 8 + grp; p < npix; p += (int64_t)gridDim.x * 8) {
    const int xx = (int)(p % g.W);
    const int64_t t = p / g.W;
    const int yy = (int)(t % g.H);
    const int n = (int)(t / g.H);
    float acc = 0.f;
    for (int tap = 0; tap < KK; ++tap) {
      const int iy = yy + tap / g.K - g.pad, ix = xx + tap % g.K - g.pad;
      if (iy < 0 || iy >= g.H || ix < 0 || ix >= g.W) continue;
      const float4* src = reinterpret_cast<const float4*>(x + (((int64_t)n * g.H + iy) * g.W + ix) * g.C);
      const float4* wr = reinterpret_cast<const float4*>(wT + tap * g.C);
      for (int c4 = sub; c4 < C4; c4 += 32) {
        const float4 v = src[c4], ww = wr[c4];
        acc = fmaf(v.x, ww.x, fmaf(v.y, ww.y, fmaf(v.z, ww.z, fmaf(v.w, ww.w, acc))));
      }
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 32);
    if (sub == 0) y[p] = acc + bias;
  }
}

// dx[n,y,x,c] = sum_tap dy[n, y - ky + pad, x - kx + pad] * w[c][ky][kx]
__global__ __launch_bounds__(HC_THREADS) void headconv_dgrad_kernel(const float* __restrict__ dy,
                                                                    const float* __restrict__ w,
                                                                    float* __restrict__ dx, HcGeom g) {
  __shared__ __attribute__((aligned(16))) float wT[9 * HC_MAXC];
  stage_wT(wT, w, g);
  __syncthreads();
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
    for (int tap = 0; tap < KK; ++tap) {
      const int oy = yy - tap / g.K + g.pad, ox = xx - tap % g.K + g.pad;
      if (oy < 0 || oy >= g.H || ox < 0 || ox >= g.W) continue;
      const float d = dy[((int64_t)n * g.H + oy) * g.W + ox];
      const float4 ww = reinterpret_cast<const float4*>(wT + tap * g.C)[c4];
      acc.x = fmaf(d, ww.x, acc.x); acc.y = fmaf(d, ww.y, acc.y);
      acc.z = fmaf(d, ww.z, acc.z); acc.w = fmaf(d, ww.w, acc.w);
    }
    reinterpret_cast<float4*>(dx)[e] = acc;
  }
}

// per-block partial[blk][tap*C + c] = sum over the block's pixels of dy[p] * x[p + tap][c]
// (+ partial[blk][KK*C] = sum dy).  32 lanes own channel quads, 8 pixel rows per pass;
// the 8 rows are folded through LDS at the end.  Requires K <= 3 (9 taps in registers)
// and C <= 128.
__global__ __launch_bounds__(HC_THREADS) void headconv_wgrad_partial(const float* __restrict__ dy,
                                                                     const float* __restrict__ x,
                                                                     float* __restrict__ part, HcGeom g,
                                                                     int64_t pix_per_blk) {
  __shared__ float4 red[8][9][32];
  __shared__ float redb[8];
  const int sub = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int KK = g.K * g.K, C4 = g.C / 4;
  const int64_t npix = (int64_t)g.N * g.H * g.W;
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_blk;
  const int64_t p1 = min(npix, p0 + pix_per_blk);
  float4 acc[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) acc[tap] = make_float4(0.f, 0.f, 0.f, 0.f);
  float bsum = 0.f;
  const bool cv = sub < C4;
  for (int64_t p = p0 + grp; p < p1; p += 8) {
    const int xx = (int)(p % g.W);
    const int64_t t = p / g.W;
    const int yy = (int)(t % g.H);
    const int n = (int)(t / g.H);
    const float d = dy[p];
    bsum += d;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap >= KK) break;
      const int iy = yy + tap / g.K - g.pad, ix = xx + tap % g.K - g.pad;
      if (!cv || iy < 0 || iy >= g.H || ix < 0 || ix >= g.W) continue;
      const float4 v = reinterpret_cast<const float4*>(x + (((int64_t)n * g.H + iy) * g.W + ix) * g.C)[sub];
      acc[tap].x = fmaf(d, v.x, acc[tap].x); acc[tap].y = fmaf(d, v.y, acc[tap].y);
      acc[tap].z = fmaf(d, v.z, acc[tap].z); acc[tap].w = fmaf(d, v.w, acc[tap].w);
    }
  }
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) red[grp][tap][sub] = acc[tap];
  if (sub == 0) redb[grp] = bsum;
  __syncthreads();
  float* P = part + (int64_t)blockIdx.x * (KK * g.C + 1);
  for (int e = threadIdx.x; e < KK * C4; e += HC_THREADS) {
    const int tap = e / C4, c4 = e % C4;
    float4 s4 = red[0][tap][c4];
    for (int r = 1; r < 8; ++r) {
      const float4 o = red[r][tap][c4];
      s4.x += o.x; s4.y += o.y; s4.z += o.z; s4.w += o.w;
    }
    float* o = P + tap * g.C + 4 * c4;
    o[0] = s4.x; o[1] = s4.y; o[2] = s4.z; o[3] = s4.w;
  }
  if (threadIdx.x == 0) {
    float s1 = 0.f;
    for (int r = 0; r < 8; ++r) s1 += redb[r];
    P[KK * g.C] = s1;
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
static int64_t hc_pix_per_blk(int64_t npix) { return cdiv(npix, 1024); }

}  // namespace mdemi

using namespace mdemi;

static int hc_check(int32_t N, int32_t H, int32_t W, int32_t C, int32_t K, int32_t pad) {
  MDEMI_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0 && C <= 128 && K > 0 && K <= 3 && pad >= 0 &&
                    2 * pad == K - 1,
                "headconv: needs C %% 4 == 0, C <= 128, K <= 3 and 'same' padding (C=%d K=%d pad=%d)", C, K, pad);
  return MDEMI_OK;
}

extern "C" int mdemi_headconv_fwd(const float* x, const float* w, const float* b, float* y, int32_t N, int32_t H,
                                  int32_t W, int32_t C, int32_t K, int32_t pad, void* stream) {
  MDEMI_REQUIRE(x && w && y, "headconv_fwd: null pointer");
  int rc = hc_check(N, H, W, C, K, pad);
  if (rc) return rc;
  HcGeom g{N, H, W, C, K, pad};
  const int64_t npix = (int64_t)N * H * W;
  hipLaunchKernelGGL(headconv_fwd_kernel, dim3(hc_grid(npix, 8 * 4)), dim3(HC_THREADS), 0,
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
