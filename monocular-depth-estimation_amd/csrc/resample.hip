// HBM-bound resampling and layout sweeps over NHWC activations.
//  - bilinear resize fwd/bwd: F.interpolate(mode='bilinear') as used by
//    NewCRFDepth.py:185-188 (x4, align_corners=False), uper_crf_head.py:51-55
//    (PPM, align_corners=False), unet_adaptive_bins.py:22 and
//    layer_utils.py:110-115 / decoder_v8.py:149-152 (align_corners=True).
//    Source-index arithmetic follows ATen's upsample_bilinear2d
//    (area_pixel_compute_source_index); the backward is a deterministic
//    gather that re-evaluates the same forward taps (no atomics).
//  - adaptive average pooling (uper_crf_head.py:38)
//  - PixelShuffle as an NHWC index map (NewCRFDepth.py:132-136)
//  - patchify for stride==kernel convs (swin_transformer.py:420-436)
//  - NCHW <-> NHWC at the model boundary
#include "common.h"

namespace mdemi {

struct Axis {
  int in, out, align;
  float scale;  // ATen rheight/rwidth
  __device__ __forceinline__ void tap(int o, int& i0, int& ip, float& l1) const {
    float src;
    if (align) src = scale * (float)o;
    else {
      src = scale * ((float)o + 0.5f) - 0.5f;
      src = src < 0.f ? 0.f : src;
    }
    i0 = (int)src;
    ip = (i0 < in - 1) ? 1 : 0;
    l1 = src - (float)i0;
  }
};

static Axis make_axis(int in, int out, int align, float user_scale) {
  Axis a;
  a.in = in; a.out = out; a.align = align;
  if (align) a.scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  else a.scale = user_scale > 0.f ? 1.f / user_scale : (float)in / (float)out;
  return a;
}

template <int VEC>
__global__ __launch_bounds__(256) void bilinear_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int N,
                                                           int C, Axis ah, Axis aw, int64_t in_cs, int64_t out_cs) {
  const int CV = C / VEC;
  const int64_t total = (int64_t)N * ah.out * aw.out * CV;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(e % CV);
    int64_t t = e / CV;
    const int ox = (int)(t % aw.out); t /= aw.out;
    const int oy = (int)(t % ah.out);
    const int n = (int)(t / ah.out);
    int h1, hp, w1, wp; float hl1, wl1;
    ah.tap(oy, h1, hp, hl1);
    aw.tap(ox, w1, wp, wl1);
    const float hl0 = 1.f - hl1, wl0 = 1.f - wl1;
    const float* base = x + ((int64_t)n * ah.in * aw.in) * in_cs + cv * VEC;
    const float* p00 = base + ((int64_t)h1 * aw.in + w1) * in_cs;
    const float* p01 = p00 + wp * in_cs;
    const float* p10 = p00 + (int64_t)hp * aw.in * in_cs;
    const float* p11 = p10 + wp * in_cs;
    float* dst = y + (((int64_t)n * ah.out + oy) * aw.out + ox) * out_cs + cv * VEC;
    if (VEC == 4) {
      const float4 a = *reinterpret_cast<const float4*>(p00), b = *reinterpret_cast<const float4*>(p01);
      const float4 c = *reinterpret_cast<const float4*>(p10), d = *reinterpret_cast<const float4*>(p11);
      float4 o;
      o.x = hl0 * (wl0 * a.x + wl1 * b.x) + hl1 * (wl0 * c.x + wl1 * d.x);
      o.y = hl0 * (wl0 * a.y + wl1 * b.y) + hl1 * (wl0 * c.y + wl1 * d.y);
      o.z = hl0 * (wl0 * a.z + wl1 * b.z) + hl1 * (wl0 * c.z + wl1 * d.z);
      o.w = hl0 * (wl0 * a.w + wl1 * b.w) + hl1 * (wl0 * c.w + wl1 * d.w);
      *reinterpret_cast<float4*>(dst) = o;
    } else {
      dst[0] = hl0 * (wl0 * p00[0] + wl1 * p01[0]) + hl1 * (wl0 * p10[0] + wl1 * p11[0]);
    }
  }
}

// conservative range of output indices whose taps can touch input index i
__device__ __forceinline__ void out_range(const Axis& a, int i, int& lo, int& hi) {
  if (a.scale <= 0.f) { lo = 0; hi = a.out - 1; return; }
  float flo, fhi;
  if (a.align) { flo = (float)(i - 1) / a.scale; fhi = (float)(i + 1) / a.scale; }
  else { flo = ((float)i - 0.5f) / a.scale - 0.5f; fhi = ((float)i + 1.5f) / a.scale - 0.5f; }
  lo = (int)floorf(flo) - 2;
  hi = (int)ceilf(fhi) + 2;
  lo = lo < 0 ? 0 : lo;
  hi = hi > a.out - 1 ? a.out - 1 : hi;
}

template <int VEC>
__global__ __launch_bounds__(256) void bilinear_bwd_kernel(const float* __restrict__ dy, float* __restrict__ dx, int N,
                                                           int C, Axis ah, Axis aw, int64_t dy_cs, int64_t dx_cs,
                                                           int accumulate) {
  const int CV = C / VEC;
  const int64_t total = (int64_t)N * ah.in * aw.in * CV;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(e % CV);
    int64_t t = e / CV;
    const int ix = (int)(t % aw.in); t /= aw.in;
    const int iy = (int)(t % ah.in);
    const int n = (int)(t / ah.in);
    int ylo, yhi, xlo, xhi;
    out_range(ah, iy, ylo, yhi);
    out_range(aw, ix, xlo, xhi);
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
    for (int oy = ylo; oy <= yhi; ++oy) {
      int h1, hp; float hl1;
      ah.tap(oy, h1, hp, hl1);
      float wy = 0.f;
      if (h1 == iy) wy += 1.f - hl1;
      if (h1 + hp == iy) wy += hl1;
      if (wy == 0.f) continue;
      for (int ox = xlo; ox <= xhi; ++ox) {
        int w1, wp; float wl1;
        aw.tap(ox, w1, wp, wl1);
        float wx = 0.f;
        if (w1 == ix) wx += 1.f - wl1;
        if (w1 + wp == ix) wx += wl1;
        if (wx == 0.f) continue;
        const float wgt = wy * wx;
        const float* src = dy + (((int64_t)n * ah.out + oy) * aw.out + ox) * dy_cs + cv * VEC;
        float sv[VEC];
        if constexpr (VEC == 4) {  // one 16-B load per tap (strides are multiples of 4 floats)
          const float4 q = *reinterpret_cast<const float4*>(src);
          sv[0] = q.x; sv[1] = q.y; sv[2] = q.z; sv[3] = q.w;
        } else {
#pragma unroll
          for (int v = 0; v < VEC; ++v) sv[v] = src[v];
        }
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] = fmaf(wgt, sv[v], acc[v]);
      }
    }
    float* dst = dx + (((int64_t)n * ah.in + iy) * aw.in + ix) * dx_cs + cv * VEC;
    if constexpr (VEC == 4) {
      float4 o = make_float4(acc[0], acc[1], acc[2], acc[3]);
      if (accumulate) {
        const float4 d = *reinterpret_cast<const float4*>(dst);
        o.x += d.x; o.y += d.y; o.z += d.z; o.w += d.w;
      }
      *reinterpret_cast<float4*>(dst) = o;
    } else {
#pragma unroll
      for (int v = 0; v < VEC; ++v) dst[v] = accumulate ? dst[v] + acc[v] : acc[v];
    }
  }
}

__global__ void adaptive_avgpool_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int H, int W,
                                            int C, int OH, int OW) {
  const int64_t total = (int64_t)N * OH * OW * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    int64_t t = e / C;
    const int ox = (int)(t % OW); t /= OW;
    const int oy = (int)(t % OH);
    const int n = (int)(t / OH);
    const int y0 = (oy * H) / OH, y1 = ((oy + 1) * H + OH - 1) / OH;
    const int x0 = (ox * W) / OW, x1 = ((ox + 1) * W + OW - 1) / OW;
    float s = 0.f;
    for (int yy = y0; yy < y1; ++yy)
      for (int xx = x0; xx < x1; ++xx) s += x[(((int64_t)n * H + yy) * W + xx) * C + c];
    y[e] = s / (float)((y1 - y0) * (x1 - x0));
  }
}

__global__ void adaptive_avgpool_bwd_kernel(const float* __restrict__ dy, float* __restrict__ dx, int N, int H, int W,
                                            int C, int OH, int OW) {
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    int64_t t = e / C;
    const int xx = (int)(t % W); t /= W;
    const int yy = (int)(t % H);
    const int n = (int)(t / H);
    float s = 0.f;
    for (int oy = 0; oy < OH; ++oy) {
      const int y0 = (oy * H) / OH, y1 = ((oy + 1) * H + OH - 1) / OH;
      if (yy < y0 || yy >= y1) continue;
      for (int ox = 0; ox < OW; ++ox) {
        const int x0 = (ox * W) / OW, x1 = ((ox + 1) * W + OW - 1) / OW;
        if (xx < x0 || xx >= x1) continue;
        s += dy[(((int64_t)n * OH + oy) * OW + ox) * C + c] / (float)((y1 - y0) * (x1 - x0));
      }
    }
    dx[e] = s;
  }
}

// PixelShuffle(r) in NHWC: y[n, y*r+i, x*r+j, c] = x[n, y, x, c*r*r + i*r + j]
// inverse = its adjoint (pixel unshuffle), used for the backward.
__global__ void pixel_shuffle_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int H, int W, int C,
                                     int r, int inverse) {
  const int OC = C / (r * r), OH = H * r, OW = W * r;
  const int64_t total = (int64_t)N * OH * OW * OC;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % OC);
    int64_t t = e / OC;
    const int X = (int)(t % OW); t /= OW;
    const int Y = (int)(t % OH);
    const int n = (int)(t / OH);
    const int yy = Y / r, i = Y % r, xx = X / r, j = X % r;
    const int64_t src = (((int64_t)n * H + yy) * W + xx) * C + c * r * r + i * r + j;
    if (!inverse) y[e] = x[src];
    else y[src] = x[e];
  }
}

// cols[(n*Hp + py)*Wp + px][(c*p + ky)*p + kx] = img[n, c, py*p+ky, px*p+kx] (zero past H/W)
__global__ void patchify_kernel(const float* __restrict__ img, float* __restrict__ cols, int N, int C, int H, int W,
                                int p) {
  const int Hp = (H + p - 1) / p, Wp = (W + p - 1) / p;
  const int K = C * p * p;
  const int64_t total = (int64_t)N * Hp * Wp * K;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % K);
    int64_t t = e / K;
    const int px = (int)(t % Wp); t /= Wp;
    const int py = (int)(t % Hp);
    const int n = (int)(t / Hp);
    const int kx = k % p, ky = (k / p) % p, c = k / (p * p);
    const int yy = py * p + ky, xx = px * p + kx;
    cols[e] = (yy < H && xx < W) ? img[(((int64_t)n * C + c) * H + yy) * W + xx] : 0.f;
  }
}

// tiled transpose of each image: [rows][cols] -> [cols][rows]
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                        int64_t rows, int64_t cols) {
  __shared__ float tile[32][33];
  const int n = blockIdx.z;
  const float* X = x + (int64_t)n * rows * cols;
  float* Y = y + (int64_t)n * rows * cols;
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int64_t r = r0 + k, c = c0 + tx;
    tile[k][tx] = (r < rows && c < cols) ? X[r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int64_t c = c0 + k, r = r0 + tx;
    if (r < rows && c < cols) Y[c * rows + r] = tile[tx][k];
  }
}

static int grid_for(int64_t total) {
  const int64_t nb = cdiv(total, 256);
  return (int)(nb < 8192 ? (nb < 1 ? 1 : nb) : 8192);
}

}  // namespace mdemi

using namespace mdemi;

extern "C" int mdemi_bilinear_fwd(const float* x, float* out, int32_t N, int32_t H, int32_t W, int32_t C, int32_t OH,
                                  int32_t OW, int32_t align_corners, float scale_h, float scale_w,
                                  int64_t in_cstride, int64_t out_cstride, void* stream) {
  MDEMI_REQUIRE(x && out && N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0, "bilinear_fwd: bad args");
  if (in_cstride <= 0) in_cstride = C;
  if (out_cstride <= 0) out_cstride = C;
  const Axis ah = make_axis(H, OH, align_corners, scale_h), aw = make_axis(W, OW, align_corners, scale_w);
  hipStream_t st = (hipStream_t)stream;
  const bool v4 = C % 4 == 0 && in_cstride % 4 == 0 && out_cstride % 4 == 0 && ((uintptr_t)x & 15) == 0 &&
                  ((uintptr_t)out & 15) == 0;
  const int64_t total = (int64_t)N * OH * OW * (v4 ? C / 4 : C);
  if (v4)
    hipLaunchKernelGGL(bilinear_fwd_kernel<4>, dim3(grid_for(total)), dim3(256), 0, st, x, out, N, C, ah, aw,
                       in_cstride, out_cstride);
  else
    hipLaunchKernelGGL(bilinear_fwd_kernel<1>, dim3(grid_for(total)), dim3(256), 0, st, x, out, N, C, ah, aw,
                       in_cstride, out_cstride);
  return check_launch("bilinear_fwd");
}

extern "C" int mdemi_bilinear_bwd(const float* dout, float* dx, int32_t N, int32_t H, int32_t W, int32_t C,
                                  int32_t OH, int32_t OW, int32_t align_corners, float scale_h, float scale_w,
                                  int64_t dout_cstride, int64_t dx_cstride, int32_t accumulate, void* stream) {
  MDEMI_REQUIRE(dout && dx && N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0, "bilinear_bwd: bad args");
  if (dout_cstride <= 0) dout_cstride = C;
  if (dx_cstride <= 0) dx_cstride = C;
  const Axis ah = make_axis(H, OH, align_corners, scale_h), aw = make_axis(W, OW, align_corners, scale_w);
  hipStream_t st = (hipStream_t)stream;
  const bool v4 = C % 4 == 0 && dout_cstride % 4 == 0 && dx_cstride % 4 == 0 && ((uintptr_t)dout & 15) == 0 &&
                  ((uintptr_t)dx & 15) == 0;
  const int64_t total = (int64_t)N * H * W * (v4 ? C / 4 : C);
  if (v4)
    hipLaunchKernelGGL(bilinear_bwd_kernel<4>, dim3(grid_for(total)), dim3(256), 0, st, dout, dx, N, C, ah, aw,
                       dout_cstride, dx_cstride, accumulate);
  else
    hipLaunchKernelGGL(bilinear_bwd_kernel<1>, dim3(grid_for(total)), dim3(256), 0, st, dout, dx, N, C, ah, aw,
                       dout_cstride, dx_cstride, accumulate);
  return check_launch("bilinear_bwd");
}

extern "C" int mdemi_adaptive_avgpool_fwd(const float* x, float* y, int32_t N, int32_t H, int32_t W, int32_t C,
                                          int32_t OH, int32_t OW, void* stream) {
  MDEMI_REQUIRE(x && y && N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0, "avgpool_fwd: bad args");
  const int64_t total = (int64_t)N * OH * OW * C;
  hipLaunchKernelGGL(adaptive_avgpool_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, y, N,
                     H, W, C, OH, OW);
  return check_launch("adaptive_avgpool_fwd");
}

extern "C" int mdemi_adaptive_avgpool_bwd(const float* dy, float* dx, int32_t N, int32_t H, int32_t W, int32_t C,
                                          int32_t OH, int32_t OW, void* stream) {
  MDEMI_REQUIRE(dy && dx && N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0, "avgpool_bwd: bad args");
  const int64_t total = (int64_t)N * H * W * C;
  hipLaunchKernelGGL(adaptive_avgpool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, dy, dx, N,
                     H, W, C, OH, OW);
  return check_launch("adaptive_avgpool_bwd");
}

extern "C" int mdemi_pixel_shuffle_nhwc(const float* x, float* y, int32_t N, int32_t H, int32_t W, int32_t C,
                                        int32_t r, int32_t inverse, void* stream) {
  MDEMI_REQUIRE(x && y && N > 0 && H > 0 && W > 0 && r > 0 && C % (r * r) == 0, "pixel_shuffle: bad args");
  const int64_t total = (int64_t)N * H * W * C;
  hipLaunchKernelGGL(pixel_shuffle_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, y, N, H, W, C,
                     r, inverse);
  return check_launch("pixel_shuffle");
}

extern "C" int mdemi_patchify_nchw(const float* img, float* cols, int32_t N, int32_t C, int32_t H, int32_t W,
                                   int32_t p, int32_t inverse, void* stream) {
  MDEMI_REQUIRE(img && cols && N > 0 && C > 0 && H > 0 && W > 0 && p > 0, "patchify: bad args");
  if (inverse) { set_error("patchify: inverse (col2im) not built"); return MDEMI_EUNSUP; }
  const int64_t total = (int64_t)N * ((H + p - 1) / p) * ((W + p - 1) / p) * C * p * p;
  hipLaunchKernelGGL(patchify_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, img, cols, N, C, H, W,
                     p);
  return check_launch("patchify");
}

static int launch_transpose(const float* x, float* y, int32_t N, int64_t rows, int64_t cols, void* stream) {
  dim3 grid((unsigned)cdiv(cols, 32), (unsigned)cdiv(rows, 32), (unsigned)N);
  MDEMI_REQUIRE(grid.y <= 65535 && grid.z <= 65535, "transpose: grid too large");
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, y, rows, cols);
  return check_launch("transpose");
}

extern "C" int mdemi_nchw_to_nhwc(const float* x, float* y, int32_t N, int32_t C, int64_t HW, void* stream) {
  MDEMI_REQUIRE(x && y && N > 0 && C > 0 && HW > 0, "nchw_to_nhwc: bad args");
  return launch_transpose(x, y, N, C, HW, stream);
}

extern "C" int mdemi_nhwc_to_nchw(const float* x, float* y, int32_t N, int32_t C, int64_t HW, void* stream) {
  MDEMI_REQUIRE(x && y && N > 0 && C > 0 && HW > 0, "nhwc_to_nchw: bad args");
  return launch_transpose(x, y, N, HW, C, stream);
}

// ---------------------------------------------------------------------------
// PatchMerging gather (swin_transformer.py:272-284): y[b,i,j] = cat(x[2i,2j],
// x[2i+1,2j], x[2i,2j+1], x[2i+1,2j+1]) with zero padding for odd H/W; the
// inverse is its adjoint (the backward), dropping the pad positions.
// ---------------------------------------------------------------------------
namespace mdemi {
__global__ void space_to_depth2_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int H, int W,
                                       int C, int inverse) {
  const int OH = (H + 1) / 2, OW = (W + 1) / 2;
  const int C4 = C / 4;
  const int64_t total = (int64_t)N * OH * OW * 4 * C4;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c4 = (int)(e % C4);
    int64_t t = e / C4;
    const int q = (int)(t % 4); t /= 4;
    const int j = (int)(t % OW); t /= OW;
    const int i = (int)(t % OH);
    const int n = (int)(t / OH);
    const int yy = 2 * i + (q & 1), xx = 2 * j + (q >> 1);
    float4* dst = reinterpret_cast<float4*>(y) + e;
    const bool in = yy < H && xx < W;
    const int64_t src = ((((int64_t)n * H + yy) * W + xx) * C) / 4 + c4;
    if (!inverse) *dst = in ? reinterpret_cast<const float4*>(x)[src] : make_float4(0.f, 0.f, 0.f, 0.f);
    else if (in) reinterpret_cast<float4*>(const_cast<float*>(x))[src] = *dst;
  }
}
}  // namespace mdemi

extern "C" int mdemi_space_to_depth2(const float* x, float* y, int32_t N, int32_t H, int32_t W, int32_t C,
                                     int32_t inverse, void* stream) {
  MDEMI_REQUIRE(x && y && N > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0, "space_to_depth2: bad args");
  const int64_t total = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2) * C;
  // inverse: x is the destination (dx), y the source (dy)
  hipLaunchKernelGGL(space_to_depth2_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, y, N, H, W,
                     C, inverse);
  return check_launch("space_to_depth2");
}

// 2-D strided copy (channel-slice concat / split of NHWC maps)
namespace mdemi {
template <int VEC>
__global__ void copy2d_kernel(const float* __restrict__ src, int64_t sld, float* __restrict__ dst, int64_t dld,
                              int64_t rows, int64_t cols, int accumulate) {
  const int64_t cv = cols / VEC;
  const int64_t total = rows * cv;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cv, c = (e % cv) * VEC;
    if (VEC == 4) {
      float4 v = *reinterpret_cast<const float4*>(src + r * sld + c);
      float4* d = reinterpret_cast<float4*>(dst + r * dld + c);
      if (accumulate) { const float4 o = *d; v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w; }
      *d = v;
    } else {
      const float v = src[r * sld + c];
      dst[r * dld + c] = accumulate ? dst[r * dld + c] + v : v;
    }
  }
}
}  // namespace mdemi

extern "C" int mdemi_copy2d(const float* src, int64_t src_ld, float* dst, int64_t dst_ld, int64_t rows, int64_t cols,
                            int32_t accumulate, void* stream) {
  // src_ld == 0 broadcasts one source row into every destination row (positional encodings)
  MDEMI_REQUIRE(src && dst && rows > 0 && cols > 0 && (src_ld >= cols || src_ld == 0) && dst_ld >= cols,
                "copy2d: bad args");
  const bool v4 = cols % 4 == 0 && src_ld % 4 == 0 && dst_ld % 4 == 0 && ((uintptr_t)src & 15) == 0 &&
                  ((uintptr_t)dst & 15) == 0;
  hipStream_t st = (hipStream_t)stream;
  if (v4)
    hipLaunchKernelGGL(copy2d_kernel<4>, dim3(grid_for(rows * cols / 4)), dim3(256), 0, st, src, src_ld, dst, dst_ld,
                       rows, cols, accumulate);
  else
    hipLaunchKernelGGL(copy2d_kernel<1>, dim3(grid_for(rows * cols)), dim3(256), 0, st, src, src_ld, dst, dst_ld, rows,
                       cols, accumulate);
  return check_launch("copy2d");
}
