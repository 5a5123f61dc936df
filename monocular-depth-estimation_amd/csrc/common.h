// Shared helpers for the mdemi gfx950 kernels: error reporting for the C ABI,
// wave64 reductions, vector types.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include "mdemi.h"

namespace mdemi {

void set_error(const char* fmt, ...);

// Launch-status check used by every entry point after its last launch.
inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return MDEMI_ELAUNCH;
  }
  return MDEMI_OK;
}

#define MDEMI_REQUIRE(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::mdemi::set_error(__VA_ARGS__);      \
      return MDEMI_EINVAL;                  \
    }                                       \
  } while (0)

// ---- wave64 reductions (DPP/shuffle through __shfl_xor over all 64 lanes) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block reduction for blockDim.x == NT (multiple of 64); `red` holds NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

// Exact-erf GELU (nn.GELU default) via Abramowitz & Stegun 7.1.26:
// erfc(z) = t(a1 + t(a2 + t(a3 + t(a4 + t a5)))) e^{-z^2}, t = 1/(1 + p z), |err| <= 1.5e-7,
// branch-free; Phi(x) is formed without cancellation for x < 0 and the
// e^{-x^2/2} factor is shared with GELU'(x) = Phi(x) + x phi(x).
__device__ __forceinline__ float gelu_cdf(float x, float& e) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  e = __expf(-z * z);
  const float half_erfc = 0.5f * poly * e;
  return x >= 0.f ? 1.f - half_erfc : half_erfc;
}
__device__ __forceinline__ float gelu_f(float x) {
  float e;
  return x * gelu_cdf(x, e);
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  float e;
  const float cdf = gelu_cdf(x, e);
  return fmaf(x * 0.39894228040143268f, e, cdf);
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float silu_f(float x) { return x * sigmoid_f(x); }
__device__ __forceinline__ float silu_grad_f(float x) {
  const float s = sigmoid_f(x);
  return fmaf(x * s, 1.f - s, s);
}

__device__ __forceinline__ float apply_act(int act, float v) {
  switch (act) {
    case MDEMI_ACT_GELU: return gelu_f(v);
    case MDEMI_ACT_RELU: return v > 0.f ? v : 0.f;
    case MDEMI_ACT_LEAKY: return v > 0.f ? v : 0.01f * v;
    case MDEMI_ACT_SIGMOID: return sigmoid_f(v);
    case MDEMI_ACT_SILU: return silu_f(v);
    default: return v;
  }
}
// derivative of act expressed through the pre-activation x (and/or output y)
__device__ __forceinline__ float act_grad(int act, float x, float y) {
  switch (act) {
    case MDEMI_ACT_GELU: return gelu_grad_f(x);
    case MDEMI_ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case MDEMI_ACT_LEAKY: return x > 0.f ? 1.f : 0.01f;
    case MDEMI_ACT_SIGMOID: return y * (1.f - y);
    case MDEMI_ACT_SILU: return silu_grad_f(x);
    default: return 1.f;
  }
}

// epilogue multipliers of the *_GRAD codes: act'(aux)
__device__ __forceinline__ bool is_grad_act(int act) {
  return act == MDEMI_ACT_GELU_GRAD || act == MDEMI_ACT_RELU_GRAD || act == MDEMI_ACT_SILU_GRAD;
}
__device__ __forceinline__ float aux_grad(int act, float a) {
  switch (act) {
    case MDEMI_ACT_GELU_GRAD: return gelu_grad_f(a);
    case MDEMI_ACT_RELU_GRAD: return a > 0.f ? 1.f : 0.f;
    default: return silu_grad_f(a);
  }
}

// Inverted dropout's keep test: element ctr kept when uniform01(seed, ctr) >= p, u from a
// splitmix64 finalizer of (seed, ctr) -- one definition for the dropout sweeps (heads.hip),
// the GEMM epilogue's fused dropout and the softmax sweep's dropped bf16 copy, so every
// form of the mask agrees bit for bit.
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t ctr) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (ctr + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(uint32_t)(z >> 40) * (1.f / 16777216.f);
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Deterministic column sum of a row-major [rows][cols] matrix (row pitch ld):
// out[c] (+)= sum_r x[r][c].  Used for bias gradients and for every
// "per-block partial rows" reduction in the library.  ws: colsum_ws_bytes().
size_t colsum_ws_bytes(int64_t rows, int64_t cols);
int colsum_launch(const float* x, int64_t rows, int64_t cols, int64_t ld, float* out, int accumulate, void* ws,
                  hipStream_t st);
// as colsum_launch, columns >= split_col going to out2[c - split_col]
int colsum_launch_split(const float* x, int64_t rows, int64_t cols, int64_t ld, float* out, float* out2,
                        int64_t split_col, int accumulate, void* ws, hipStream_t st);
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace mdemi
