// Conv weight re-layouts between the reference's [Cout][Cin][KH][KW] parameters
// and the GEMM operand images the NHWC implicit-GEMM convs consume (one pass
// per call, one thread per output element; weights are small, so this is a
// launch-latency-sized HBM sweep: 8 B per element).
//   MDEMI_WL_OHWI  : out[co][ky][kx][c] = w[co][c][ky][kx]          (fwd / patch dgrad)
//   MDEMI_WL_OIHW  : out[co][c][ky][kx] = w[co][ky][kx][c]          (wgrad back to the parameter)
//   MDEMI_WL_DGRAD : out[ky][kx][co][c] = w[co][c][KH-1-ky][KW-1-kx] (dX = conv(dY, flip(W)^T))
#include "common.h"
#include "mdemi_ext.h"

namespace mdemi {

// out16 (optional): the RNE bf16 copy of each re-laid-out element (a bf16 conv GEMM's operand)
__global__ void __launch_bounds__(256) conv_wlayout_kernel(const float* __restrict__ w, float* __restrict__ out,
                                                           __bf16* __restrict__ out16, int cout, int cin, int kh,
                                                           int kw, int mode) {
  const int64_t n = (int64_t)cout * cin * kh * kw;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = t;
    int64_t src;
    if (mode == MDEMI_WL_OHWI) {  // t = ((co*kh + ky)*kw + kx)*cin + c
      const int c = (int)(r % cin); r /= cin;
      const int kx = (int)(r % kw); r /= kw;
      const int ky = (int)(r % kh);
      const int co = (int)(r / kh);
      src = (((int64_t)co * cin + c) * kh + ky) * kw + kx;
    } else if (mode == MDEMI_WL_OIHW) {  // t = ((co*cin + c)*kh + ky)*kw + kx
      const int kx = (int)(r % kw); r /= kw;
      const int ky = (int)(r % kh); r /= kh;
      const int c = (int)(r % cin);
      const int co = (int)(r / cin);
      src = (((int64_t)co * kh + ky) * kw + kx) * cin + c;
    } else {  // t = ((ky*kw + kx)*cout + co)*cin + c
      const int c = (int)(r % cin); r /= cin;
      const int co = (int)(r % cout); r /= cout;
      const int kx = (int)(r % kw);
      const int ky = (int)(r / kw);
      src = (((int64_t)co * cin + c) * kh + (kh - 1 - ky)) * kw + (kw - 1 - kx);
    }
    const float v = w[src];
    out[t] = v;
    if (out16) out16[t] = (__bf16)v;
  }
}

}  // namespace mdemi

using namespace mdemi;

extern "C" int mdemi_conv_weight_layout16(const float* w, float* out, void* out16, int32_t cout, int32_t cin,
                                          int32_t kh, int32_t kw, int32_t mode, void* stream) {
  MDEMI_REQUIRE(w && out && w != out && cout > 0 && cin > 0 && kh > 0 && kw > 0 &&
                    (mode == MDEMI_WL_OHWI || mode == MDEMI_WL_OIHW || mode == MDEMI_WL_DGRAD),
                "conv_weight_layout: bad args");
  const int64_t n = (int64_t)cout * cin * kh * kw;
  const unsigned grid = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(conv_wlayout_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, w, out, (__bf16*)out16,
                     cout, cin, kh, kw, mode);
  return check_launch("conv_weight_layout");
}

extern "C" int mdemi_conv_weight_layout(const float* w, float* out, int32_t cout, int32_t cin, int32_t kh, int32_t kw,
                                        int32_t mode, void* stream) {
  return mdemi_conv_weight_layout16(w, out, nullptr, cout, cin, kh, kw, mode, stream);
}
