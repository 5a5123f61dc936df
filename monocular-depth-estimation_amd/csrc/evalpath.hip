// Evaluation-path sweeps: horizontal flip of an NCHW batch and the flip-eval
// average pred = (a + flip_w(b)) / 2 (the config key eval.flip_eval of
// json/{nyu,kitti}/*.json; run.py, which applied it, is absent from the
// reference snapshot -- restated as in upstream NeW-CRFs / AdaBins eval).
// Both are pure HBM sweeps: 8 B (flip) / 12 B (flip-average) per element.
// One thread owns 4 consecutive output columns: the mirrored source columns
// are also 4 consecutive floats, read as one float4 when the row allows it.
#include "common.h"
#include "mdemi_ext.h"

namespace mdemi {

template <bool AVG, bool VEC>
__global__ void __launch_bounds__(256) flip_w_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                     float* __restrict__ y, int64_t rows, int32_t W) {
  const int32_t q = (W + 3) >> 2;  // column quads per row
  const int64_t total = rows * q;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / q;
    const int32_t w0 = (int32_t)(i - r * q) * 4;
    const float* src = (AVG ? b : a) + r * W;
    float* dst = y + r * W;
    if (VEC) {
      // output columns w0..w0+3 read source columns W-4-w0..W-1-w0 (reversed)
      const float4 s = *reinterpret_cast<const float4*>(src + (W - 4 - w0));
      float4 o = make_float4(s.w, s.z, s.y, s.x);
      if (AVG) {
        const float4 p = *reinterpret_cast<const float4*>(a + r * W + w0);
        o = make_float4(0.5f * (p.x + o.x), 0.5f * (p.y + o.y), 0.5f * (p.z + o.z), 0.5f * (p.w + o.w));
      }
      *reinterpret_cast<float4*>(dst + w0) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t w = w0 + j;
        if (w < W) {
          const float s = src[W - 1 - w];
          dst[w] = AVG ? 0.5f * (a[r * W + w] + s) : s;
        }
      }
    }
  }
}

}  // namespace mdemi

using namespace mdemi;

static bool flip_vec(const void* p0, const void* p1, const void* p2, int32_t W) {
  auto al = [](const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; };
  return (W & 3) == 0 && al(p0) && al(p1) && al(p2);
}

static unsigned flip_grid(int64_t rows, int32_t W) {
  const int64_t work = rows * ((W + 3) / 4);
  const int64_t blocks = (work + 255) / 256;
  return (unsigned)(blocks < 8192 ? (blocks > 0 ? blocks : 1) : 8192);
}

extern "C" int mdemi_flip_w(const float* x, float* y, int64_t rows, int32_t W, void* stream) {
  MDEMI_REQUIRE(x && y && x != y && rows > 0 && W > 0, "flip_w: bad args (out-of-place only)");
  auto k = flip_vec(x, y, nullptr, W) ? flip_w_kernel<false, true> : flip_w_kernel<false, false>;
  hipLaunchKernelGGL(k, dim3(flip_grid(rows, W)), dim3(256), 0, (hipStream_t)stream, x, nullptr, y, rows, W);
  return check_launch("flip_w");
}

extern "C" int mdemi_flip_avg_w(const float* a, const float* b, float* y, int64_t rows, int32_t W, void* stream) {
  MDEMI_REQUIRE(a && b && y && y != b && rows > 0 && W > 0, "flip_avg_w: bad args (out must not alias b)");
  auto k = flip_vec(a, b, y, W) ? flip_w_kernel<true, true> : flip_w_kernel<true, false>;
  hipLaunchKernelGGL(k, dim3(flip_grid(rows, W)), dim3(256), 0, (hipStream_t)stream, a, b, y, rows, W);
  return check_launch("flip_avg_w");
}
