// Transformer-head and depth-head sweeps of the AdaBins / Depthformer-v8
// rows, and the evaluation metrics:
//  - row softmax fwd/bwd (attention probabilities: layers.py:8-9 via
//    nn.TransformerEncoderLayer, luna_layer.py:213-215,244-246,
//    self_attention.py:72-74)
//  - counter-based inverted dropout (mask recomputed in the backward)
//  - channels-last bin head: softmax over bins + centre dot
//    (unet_adaptive_bins.py:97,107; decoder_v8.py:158-159; depthformer_v8.py:73)
//  - bin widths -> edges -> centres (unet_adaptive_bins.py:99-105,
//    miniViT.py:38-46, depthformer_v8.py:62-66, decoder_v8.py:163-166)
//  - replicate-padding adjoint (layer_utils.py:18-22)
//  - masked depth metrics (utils/depth_utils.py:4-54)
// All HBM-bound; reductions are fixed-order (block partials + ordered final sums).
#include "common.h"

#include <algorithm>
#include "mdemi_ext.h"

namespace mdemi {

static unsigned grid_1d(int64_t total, int per_block = 256) {
  int64_t g = cdiv(total, per_block);
  return (unsigned)(g < 1 ? 1 : (g > 65535 * 8 ? 65535 * 8 : g));
}

// ---------------------------------------------------------------------------
// softmax: short rows (cols <= 1024) -> one wave per row, row held in registers;
// long rows -> one 256-thread block per row, two sweeps.
// ---------------------------------------------------------------------------
constexpr int SM_REG = 16;  // values per lane for the wave-per-row path

// y16 / dx16 (optional): the RNE bf16 copy of the result, for the bf16 GEMM that reads it
// (attention probabilities into P.V, the score gradient into dQ / dK; bf16 storage).
// SmDrop (seed non-null): y16 holds the dropped-out probabilities instead -- element
// (row, c) kept when uniform01(seed[0] + add, offset + row * cols + c) >= p, kept values
// times inv -- the bf16 copy mdemi_dropout_dev16 would write from y, so P.V reads it with no
// dropout sweep and no fp32 copy of the dropped probabilities (y stays the softmax).
struct SmDrop {
  const uint64_t* seed;
  uint64_t add, offset;
  float p, inv;
};
__device__ __forceinline__ float sm_drop16(const SmDrop& d, uint64_t seed, uint64_t idx, float o) {
  return d.seed ? (uniform01(seed, d.offset + idx) >= d.p ? o * d.inv : 0.f) : o;
}
__global__ __launch_bounds__(256) void softmax_wave_fwd(const float* __restrict__ x, float* __restrict__ y,
                                                        int64_t rows, int cols, float scale,
                                                        __bf16* __restrict__ y16, SmDrop dr) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * cols;
  float v[SM_REG];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < SM_REG; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < cols ? scale * xr[c] : -INFINITY;
    m = fmaxf(m, v[i]);
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < SM_REG; ++i) {
    v[i] = __expf(v[i] - m);
    s += v[i];
  }
  s = wave_sum(s);
  const float inv = 1.f / s;
  float* yr = y + row * cols;
  const uint64_t dseed = dr.seed ? dr.seed[0] + dr.add : 0;
#pragma unroll
  for (int i = 0; i < SM_REG; ++i) {
    const int c = lane + 64 * i;
    if (c < cols) {
      yr[c] = v[i] * inv;
      if (y16) y16[row * cols + c] = (__bf16)sm_drop16(dr, dseed, (uint64_t)(row * cols + c), v[i] * inv);
    }
  }
}

__global__ __launch_bounds__(256) void softmax_block_fwd(const float* __restrict__ x, float* __restrict__ y, int cols,
                                                         float scale, __bf16* __restrict__ y16, SmDrop dr) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  const float* xr = x + row * cols;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < cols; c += 256) {
    const float v = scale * xr[c];
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
    } else {
      s += __expf(v - m);
    }
  }
  // combine (m, s) across the block
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float wm = wave_max(m);
  float ws = wave_sum(m == -INFINITY ? 0.f : s * __expf(m - wm));
  if (lane == 0) {
    red[wid] = wm;
    red[4 + wid] = ws;
  }
  __syncthreads();
  float gm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float gs = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) gs += red[4 + i] * __expf(red[i] - gm);
  const float inv = 1.f / gs;
  float* yr = y + row * cols;
  const uint64_t dseed = dr.seed ? dr.seed[0] + dr.add : 0;
  for (int c = threadIdx.x; c < cols; c += 256) {
    const float o = __expf(scale * xr[c] - gm) * inv;
    yr[c] = o;
    if (y16) y16[row * cols + c] = (__bf16)sm_drop16(dr, dseed, (uint64_t)(row * cols + c), o);
  }
}

__global__ __launch_bounds__(256) void softmax_wave_bwd(const float* __restrict__ y, const float* __restrict__ dy,
                                                        float* __restrict__ dx, int64_t rows, int cols, float scale,
                                                        int accumulate, __bf16* __restrict__ dx16) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* yr = y + row * cols;
  const float* gr = dy + row * cols;
  float yv[SM_REG], gv[SM_REG];
  float d = 0.f;
#pragma unroll
  for (int i = 0; i < SM_REG; ++i) {
    const int c = lane + 64 * i;
    yv[i] = c < cols ? yr[c] : 0.f;
    gv[i] = c < cols ? gr[c] : 0.f;
    d = fmaf(yv[i], gv[i], d);
  }
  d = wave_sum(d);
  float* xr = dx + row * cols;
#pragma unroll
  for (int i = 0; i < SM_REG; ++i) {
    const int c = lane + 64 * i;
    if (c < cols) {
      const float v = scale * yv[i] * (gv[i] - d);
      const float o = accumulate ? xr[c] + v : v;
      xr[c] = o;
      if (dx16) dx16[row * cols + c] = (__bf16)o;
    }
  }
}

__global__ __launch_bounds__(256) void softmax_block_bwd(const float* __restrict__ y, const float* __restrict__ dy,
                                                         float* __restrict__ dx, int cols, float scale,
                                                         int accumulate, __bf16* __restrict__ dx16) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const float* yr = y + row * cols;
  const float* gr = dy + row * cols;
  float d = 0.f;
  for (int c = threadIdx.x; c < cols; c += 256) d = fmaf(yr[c], gr[c], d);
  d = block_sum<256>(d, red);
  float* xr = dx + row * cols;
  for (int c = threadIdx.x; c < cols; c += 256) {
    const float v = scale * yr[c] * (gr[c] - d);
    const float o = accumulate ? xr[c] + v : v;
    xr[c] = o;
    if (dx16) dx16[row * cols + c] = (__bf16)o;
  }
}

// ---------------------------------------------------------------------------
// dropout: keep(i) = uniform01(seed, offset + i) >= p (common.h)
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void dropout_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                                                      float p, float inv_keep, uint64_t seed, uint64_t offset) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = uniform01(seed, offset + (uint64_t)i) >= p ? x[i] * inv_keep : 0.f;
}

// the same mask with the seed read from device memory (seed_dev[0] + seed_add):
// a seed drawn on the GPU by the caller changes on every replay of a captured
// graph, where a host seed would be frozen into the kernel arguments
__global__ __launch_bounds__(256) void dropout_dev_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                          int64_t n, float p, float inv_keep,
                                                          const uint64_t* __restrict__ seed_dev, uint64_t seed_add,
                                                          uint64_t offset) {
  const uint64_t seed = seed_dev[0] + seed_add;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = uniform01(seed, offset + (uint64_t)i) >= p ? x[i] * inv_keep : 0.f;
}

// float4 form (n % 4 == 0, 16-B aligned): the same mask element for element, four hashes
// per thread and one 16-B load / store -- the scalar form reached ~45 % of HBM
typedef __bf16 dp_bf16x4_t __attribute__((ext_vector_type(4)));
typedef float dp_f32x4_t __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void dropout_dev4_kernel(const float4* __restrict__ x, float4* __restrict__ y,
                                                           int64_t n4, float p, float inv_keep,
                                                           const uint64_t* __restrict__ seed_dev, uint64_t seed_add,
                                                           uint64_t offset, dp_bf16x4_t* __restrict__ y16) {
  const uint64_t seed = seed_dev[0] + seed_add;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256) {
    const float4 v = x[e];
    const uint64_t i = offset + 4 * (uint64_t)e;
    float4 o;
    o.x = uniform01(seed, i) >= p ? v.x * inv_keep : 0.f;
    o.y = uniform01(seed, i + 1) >= p ? v.y * inv_keep : 0.f;
    o.z = uniform01(seed, i + 2) >= p ? v.z * inv_keep : 0.f;
    o.w = uniform01(seed, i + 3) >= p ? v.w * inv_keep : 0.f;
    y[e] = o;
    if (y16) {
      const dp_f32x4_t ov = {o.x, o.y, o.z, o.w};
      y16[e] = __builtin_convertvector(ov, dp_bf16x4_t);
    }
  }
}

__global__ __launch_bounds__(256) void act_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                                                      int act) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = apply_act(act, x[i]);
}

// ---------------------------------------------------------------------------
// channels-last bin head: one wave per pixel row of K bins (K % 4 == 0)
// ---------------------------------------------------------------------------
constexpr int BH_PIX = 64;  // pixels per wave in the backward partials

__global__ __launch_bounds__(256) void binhead_nhwc_fwd_kernel(const float* __restrict__ logits,
                                                               const float* __restrict__ centers,
                                                               float* __restrict__ pred, float* __restrict__ stats,
                                                               int64_t HW, int K, int64_t npix) {
  const int lane = threadIdx.x & 63;
  const int K4 = K >> 2;
  for (int64_t pix = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); pix < npix; pix += (int64_t)gridDim.x * 4) {
    const int64_t b = pix / HW;
    const float* lr = logits + pix * K;
    const float* cr = centers + b * K;
    float m = -INFINITY;
    for (int k4 = lane; k4 < K4; k4 += 64) {
      const float4 v = *reinterpret_cast<const float4*>(lr + 4 * k4);
      m = fmaxf(m, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
    m = wave_max(m);
    float s = 0.f, d = 0.f;
    for (int k4 = lane; k4 < K4; k4 += 64) {
      const float4 v = *reinterpret_cast<const float4*>(lr + 4 * k4);
      const float4 c = *reinterpret_cast<const float4*>(cr + 4 * k4);
      const float e0 = __expf(v.x - m), e1 = __expf(v.y - m), e2 = __expf(v.z - m), e3 = __expf(v.w - m);
      s += (e0 + e1) + (e2 + e3);
      d = fmaf(e0, c.x, fmaf(e1, c.y, fmaf(e2, c.z, fmaf(e3, c.w, d))));
    }
    s = wave_sum(s);
    d = wave_sum(d);
    if (lane == 0) {
      const float inv = 1.f / s;
      pred[pix] = d * inv;
      stats[2 * pix] = m;
      stats[2 * pix + 1] = inv;
    }
  }
}

// K = 64 * NV (the 256 bins of AdaBins / Depthformer: NV = 4): 16 lanes per pixel, four
// pixels per wave, each lane holding its NV float4 of the row in registers -- the row is
// read once (the kernel above reads it twice) and the three reductions are 4-step
// shuffles within the 16-lane group instead of 6-step wave reductions per pixel.
template <int NV>
__global__ __launch_bounds__(256) void binhead_nhwc_fwd_g16(const float* __restrict__ logits,
                                                            const float* __restrict__ centers,
                                                            float* __restrict__ pred, float* __restrict__ stats,
                                                            int64_t HW, int64_t npix) {
  constexpr int K = 64 * NV;
  const int gl = threadIdx.x & 15;  // lane within the pixel's group
  const int64_t groups = (int64_t)gridDim.x * 16;
  for (int64_t pix = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); pix < npix; pix += groups) {
    const int64_t b = pix / HW;
    const float4* lr = reinterpret_cast<const float4*>(logits + pix * K);
    const float4* cr = reinterpret_cast<const float4*>(centers + b * K);
    float4 v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = lr[gl + 16 * j];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NV; ++j) m = fmaxf(m, fmaxf(fmaxf(v[j].x, v[j].y), fmaxf(v[j].z, v[j].w)));
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 16));
    float s = 0.f, d = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const float4 c = cr[gl + 16 * j];
      const float e0 = __expf(v[j].x - m), e1 = __expf(v[j].y - m), e2 = __expf(v[j].z - m), e3 = __expf(v[j].w - m);
      s += (e0 + e1) + (e2 + e3);
      d = fmaf(e0, c.x, fmaf(e1, c.y, fmaf(e2, c.z, fmaf(e3, c.w, d))));
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      s += __shfl_xor(s, o, 16);
      d += __shfl_xor(d, o, 16);
    }
    if (gl == 0) {
      const float inv = 1.f / s;
      pred[pix] = d * inv;
      *reinterpret_cast<float2*>(stats + 2 * pix) = make_float2(m, inv);
    }
  }
}

// grid (chunks, B): each wave handles BH_PIX pixels of image b; dcenters partials
// per wave are combined per block and written to part[b][chunk][K].
__global__ __launch_bounds__(256) void binhead_nhwc_bwd_kernel(const float* __restrict__ logits,
                                                               const float* __restrict__ centers,
                                                               const float* __restrict__ pred,
                                                               const float* __restrict__ stats,
                                                               const float* __restrict__ dpred,
                                                               float* __restrict__ dlogits, float* __restrict__ part,
                                                               int64_t HW, int K, int nchunk) {
  extern __shared__ float sred[];  // [4][K]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b = blockIdx.y, ch = blockIdx.x;
  const int K4 = K >> 2;
  for (int i = threadIdx.x; i < 4 * K; i += 256) sred[i] = 0.f;
  __syncthreads();
  const int64_t p0 = ((int64_t)ch * 4 + wid) * BH_PIX;
  const int64_t p1 = min(HW, p0 + BH_PIX);
  const float* cr = centers + (int64_t)b * K;
  float* mine = sred + wid * K;
  for (int64_t p = p0; p < p1; ++p) {
    const int64_t pix = (int64_t)b * HW + p;
    const float m = stats[2 * pix], inv = stats[2 * pix + 1];
    const float g = dpred[pix], pr = pred[pix];
    const float* lr = logits + pix * K;
    float* dr = dlogits + pix * K;
    for (int k4 = lane; k4 < K4; k4 += 64) {
      const float4 v = *reinterpret_cast<const float4*>(lr + 4 * k4);
      const float4 c = *reinterpret_cast<const float4*>(cr + 4 * k4);
      const float q0 = __expf(v.x - m) * inv, q1 = __expf(v.y - m) * inv, q2 = __expf(v.z - m) * inv,
                  q3 = __expf(v.w - m) * inv;
      *reinterpret_cast<float4*>(dr + 4 * k4) =
          make_float4(q0 * g * (c.x - pr), q1 * g * (c.y - pr), q2 * g * (c.z - pr), q3 * g * (c.w - pr));
      float4* acc = reinterpret_cast<float4*>(mine + 4 * k4);
      float4 a = *acc;
      a.x = fmaf(q0, g, a.x); a.y = fmaf(q1, g, a.y); a.z = fmaf(q2, g, a.z); a.w = fmaf(q3, g, a.w);
      *acc = a;
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += 256)
    part[((int64_t)b * nchunk + ch) * K + k] = (sred[k] + sred[K + k]) + (sred[2 * K + k] + sred[3 * K + k]);
}

// K = 64 * NV: the backward with the forward's 16-lane groups.  Grid (chunks, B) as above
// (4 * BH_PIX pixels per block); the block's 16 groups sweep 16 consecutive pixels per
// step, so a step reads and writes 16 contiguous rows.  Each lane keeps its bins' share
// of sum_p g p_k (the dcenters partial) in registers across its pixels; the four groups
// of a wave combine by shuffles and the four waves through LDS, in a fixed order.
template <int NV>
__global__ __launch_bounds__(256) void binhead_nhwc_bwd_g16(const float* __restrict__ logits,
                                                            const float* __restrict__ centers,
                                                            const float* __restrict__ pred,
                                                            const float* __restrict__ stats,
                                                            const float* __restrict__ dpred,
                                                            float* __restrict__ dlogits, float* __restrict__ part,
                                                            int64_t HW, int nchunk) {
  constexpr int K = 64 * NV;
  __shared__ float4 red[4][K / 4];
  const int gl = threadIdx.x & 15, grp = threadIdx.x >> 4, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b = blockIdx.y, ch = blockIdx.x;
  const float4* cr = reinterpret_cast<const float4*>(centers + (int64_t)b * K);
  float4 c[NV], acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    c[j] = cr[gl + 16 * j];
    acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int64_t p0 = (int64_t)ch * 4 * BH_PIX;
  for (int it = 0; it < 4 * BH_PIX / 16; ++it) {
    const int64_t p = p0 + it * 16 + grp;
    if (p >= HW) break;
    const int64_t pix = (int64_t)b * HW + p;
    const float2 st = *reinterpret_cast<const float2*>(stats + 2 * pix);
    const float g = dpred[pix], pr = pred[pix];
    const float4* lr = reinterpret_cast<const float4*>(logits + pix * K);
    float4* dr = reinterpret_cast<float4*>(dlogits + pix * K);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const float4 v = lr[gl + 16 * j];
      const float q0 = __expf(v.x - st.x) * st.y, q1 = __expf(v.y - st.x) * st.y, q2 = __expf(v.z - st.x) * st.y,
                  q3 = __expf(v.w - st.x) * st.y;
      dr[gl + 16 * j] = make_float4(q0 * g * (c[j].x - pr), q1 * g * (c[j].y - pr), q2 * g * (c[j].z - pr),
                                    q3 * g * (c[j].w - pr));
      acc[j].x = fmaf(q0, g, acc[j].x); acc[j].y = fmaf(q1, g, acc[j].y);
      acc[j].z = fmaf(q2, g, acc[j].z); acc[j].w = fmaf(q3, g, acc[j].w);
    }
  }
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      acc[j].x += __shfl_xor(acc[j].x, o, 64); acc[j].y += __shfl_xor(acc[j].y, o, 64);
      acc[j].z += __shfl_xor(acc[j].z, o, 64); acc[j].w += __shfl_xor(acc[j].w, o, 64);
    }
  if (lane < 16)
#pragma unroll
    for (int j = 0; j < NV; ++j) red[wid][gl + 16 * j] = acc[j];
  __syncthreads();
  const float* rf = reinterpret_cast<const float*>(red);
  for (int k = threadIdx.x; k < K; k += 256)
    part[((int64_t)b * nchunk + ch) * K + k] = (rf[k] + rf[K + k]) + (rf[2 * K + k] + rf[3 * K + k]);
}

// dcenters[b][k] = sum over chunks of part[b][chunk][k]: grid (ceil(K/64), B), lane = k,
// wave w sums chunks w, w+4, ... (coalesced 256-B rows), then the 4 wave partials are
// added in a fixed order through LDS (deterministic).
__global__ __launch_bounds__(256) void binhead_nhwc_final(const float* __restrict__ part, float* __restrict__ dc,
                                                          int B, int K, int nchunk) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b = blockIdx.y, k = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (k < K) {
    const float* pb = part + (int64_t)b * nchunk * K + k;
#pragma unroll 4
    for (int i = wid; i < nchunk; i += 4) s += pb[(int64_t)i * K];
  }
  red[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && k < K) dc[(int64_t)b * K + k] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// ---------------------------------------------------------------------------
// bins: one thread per batch row (B and K are small); sequential sums keep
// the reference's left-to-right cumsum order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bins_act(int mode, float x) {
  return mode == MDEMI_BINS_RELU ? fmaxf(x, 0.f) + 0.1f : (x > 0.f ? x : 0.1f * expm1f(x)) + 0.1f;
}
__device__ __forceinline__ float bins_act_grad(int mode, float x) {
  return mode == MDEMI_BINS_RELU ? (x > 0.f ? 1.f : 0.f) : (x > 0.f ? 1.f : 0.1f * __expf(x));
}

__global__ void bins_fwd_kernel(const float* __restrict__ raw, float* __restrict__ widths_n,
                                float* __restrict__ edges, float* __restrict__ centers, int B, int K, int mode,
                                float min_val, float max_val) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* r = raw + (int64_t)b * K;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bins_act(mode, r[k]);
  const float range = max_val - min_val;
  float e = min_val;
  if (edges) edges[(int64_t)b * (K + 1)] = e;
  for (int k = 0; k < K; ++k) {
    const float wn = bins_act(mode, r[k]) / s;
    if (widths_n) widths_n[(int64_t)b * K + k] = wn;
    const float e1 = e + range * wn;
    if (edges) edges[(int64_t)b * (K + 1) + k + 1] = e1;
    centers[(int64_t)b * K + k] = 0.5f * (e + e1);
    e = e1;
  }
}

__global__ void bins_bwd_kernel(const float* __restrict__ raw, const float* __restrict__ dcenters,
                                const float* __restrict__ dedges, const float* __restrict__ dwidths,
                                float* __restrict__ draw, int B, int K, int mode, float min_val, float max_val) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* r = raw + (int64_t)b * K;
  const float* dc = dcenters + (int64_t)b * K;
  const float* de = dedges ? dedges + (int64_t)b * (K + 1) : nullptr;
  float* dr = draw + (int64_t)b * K;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bins_act(mode, r[k]);
  const float range = max_val - min_val;
  // d(width_j) = sum_{k > j} dE_k with dE_k = dedges_k + 0.5 dc_k + 0.5 dc_{k-1}; walk j downwards
  float suffix = 0.f, dot = 0.f;
  for (int j = K - 1; j >= 0; --j) {
    const int k = j + 1;
    float dE = 0.5f * dc[k - 1] + (k < K ? 0.5f * dc[k] : 0.f);
    if (de) dE += de[k];
    suffix += dE;
    const float dwn = range * suffix + (dwidths ? dwidths[(int64_t)b * K + j] : 0.f);
    dr[j] = dwn;  // temporarily d(normalised width)
    dot = fmaf(dwn, bins_act(mode, r[j]) / s, dot);
  }
  for (int j = 0; j < K; ++j) dr[j] = (dr[j] - dot) / s * bins_act_grad(mode, r[j]);
}

// ---------------------------------------------------------------------------
// replicate-padding adjoint
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pad_fold_kernel(const float* __restrict__ dxp, float* __restrict__ dx, int N,
                                                       int H, int W, int C, int p) {
  const int C4 = C >> 2, Hp = H + 2 * p, Wp = W + 2 * p;
  const int64_t total = (int64_t)N * H * W * C4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    int64_t t = e / C4;
    const int x = (int)(t % W); t /= W;
    const int y = (int)(t % H);
    const int n = (int)(t / H);
    const int ya = y == 0 ? 0 : y + p, yb = y == H - 1 ? Hp - 1 : y + p;
    const int xa = x == 0 ? 0 : x + p, xb = x == W - 1 ? Wp - 1 : x + p;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int yy = ya; yy <= yb; ++yy)
      for (int xx = xa; xx <= xb; ++xx) {
        const float4 v = *reinterpret_cast<const float4*>(dxp + (((int64_t)n * Hp + yy) * Wp + xx) * C + c4 * 4);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
    reinterpret_cast<float4*>(dx)[e] = s;
  }
}

__global__ __launch_bounds__(256) void unpatchify_kernel(const float* __restrict__ cols, float* __restrict__ x, int N,
                                                         int H, int W, int C, int p, int OH, int OW) {
  const int C4 = C >> 2;
  const int64_t total = (int64_t)N * H * W * C4;
  const int64_t K = (int64_t)p * p * C;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    int64_t t = e / C4;
    const int xx = (int)(t % W); t /= W;
    const int yy = (int)(t % H);
    const int n = (int)(t / H);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (yy < OH * p && xx < OW * p) {
      const int64_t row = ((int64_t)n * OH + yy / p) * OW + xx / p;
      v = *reinterpret_cast<const float4*>(cols + row * K + ((int64_t)(yy % p) * p + xx % p) * C + c4 * 4);
    }
    reinterpret_cast<float4*>(x)[e] = v;
  }
}

// ---------------------------------------------------------------------------
// depth metrics: grid (chunks, B); 11 sums per image
// ---------------------------------------------------------------------------
constexpr int MET_N = 11;  // count, a1, a2, a3, abs_rel, sq_rel, sq, sq_log, err, err^2, log10

__global__ __launch_bounds__(256) void metrics_partial(const float* __restrict__ pred, const float* __restrict__ gt,
                                                       double* __restrict__ part, int H, int W, int y0, int y1, int x0,
                                                       int x1, float dmin, float dmax, int clamp_pred, int nchunk) {
  __shared__ float red[MET_N][4];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int64_t HW = (int64_t)H * W;
  const int64_t per = (HW + nchunk - 1) / nchunk;
  const int64_t p0 = (int64_t)ch * per, p1 = min(HW, p0 + per);
  float acc[MET_N];
#pragma unroll
  for (int i = 0; i < MET_N; ++i) acc[i] = 0.f;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) {
    const int y = (int)(p / W), x = (int)(p % W);
    const float g = gt[(int64_t)b * HW + p];
    if (y < y0 || y >= y1 || x < x0 || x >= x1 || !(g > dmin) || !(g < dmax)) continue;
    float q = pred[(int64_t)b * HW + p];
    if (clamp_pred) q = fminf(fmaxf(q, dmin), dmax);
    const float th = fmaxf(g / q, q / g);
    const float diff = g - q;
    const float lg = logf(g), lq = logf(q);
    const float err = lq - lg;
    acc[0] += 1.f;
    acc[1] += th < 1.25f ? 1.f : 0.f;
    acc[2] += th < 1.25f * 1.25f ? 1.f : 0.f;
    acc[3] += th < 1.25f * 1.25f * 1.25f ? 1.f : 0.f;
    acc[4] += fabsf(diff) / g;
    acc[5] += diff * diff / g;
    acc[6] += diff * diff;
    acc[7] += (lg - lq) * (lg - lq);
    acc[8] += err;
    acc[9] += err * err;
    acc[10] += fabsf(log10f(g) - log10f(q));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < MET_N; ++i) {
    const float v = wave_sum(acc[i]);
    if (lane == 0) red[i][wid] = v;
  }
  __syncthreads();
  if (threadIdx.x < MET_N) {
    const int i = threadIdx.x;
    part[((int64_t)b * nchunk + ch) * MET_N + i] =
        ((double)red[i][0] + (double)red[i][1]) + ((double)red[i][2] + (double)red[i][3]);
  }
}

__global__ void metrics_final(const double* __restrict__ part, double* __restrict__ out, int B, int nchunk) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s[MET_N];
  for (int i = 0; i < MET_N; ++i) s[i] = 0.0;
  for (int c = 0; c < nchunk; ++c)
    for (int i = 0; i < MET_N; ++i) s[i] += part[((int64_t)b * nchunk + c) * MET_N + i];
  const double n = s[0];
  double* o = out + (int64_t)b * 10;
  const double inv = n > 0 ? 1.0 / n : 0.0;
  o[0] = s[1] * inv;
  o[1] = s[2] * inv;
  o[2] = s[3] * inv;
  o[3] = s[4] * inv;
  o[4] = s[5] * inv;
  o[5] = sqrt(s[6] * inv);
  o[6] = sqrt(s[7] * inv);
  const double me = s[8] * inv;
  o[7] = sqrt(fmax(s[9] * inv - me * me, 0.0)) * 100.0;
  o[8] = s[10] * inv;
  o[9] = n;
}

static int metrics_chunks(int64_t HW) {
  int64_t c = cdiv(HW, 4096);
  return (int)(c < 1 ? 1 : (c > 256 ? 256 : c));
}

}  // namespace mdemi

using namespace mdemi;

extern "C" int mdemi_softmax_fwd(const float* x, float* y, int64_t rows, int32_t cols, float scale, void* stream) {
  return mdemi_softmax_fwd16(x, y, nullptr, rows, cols, scale, stream);
}

static int softmax_fwd_launch(const float* x, float* y, void* y16, int64_t rows, int32_t cols, float scale,
                              const SmDrop& dr, hipStream_t st) {
  if (cols <= 64 * SM_REG)
    hipLaunchKernelGGL(softmax_wave_fwd, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, st, x, y, rows, cols, scale,
                       (__bf16*)y16, dr);
  else
    hipLaunchKernelGGL(softmax_block_fwd, dim3((unsigned)rows), dim3(256), 0, st, x, y, cols, scale, (__bf16*)y16,
                       dr);
  return check_launch("softmax_fwd");
}

extern "C" int mdemi_softmax_fwd16(const float* x, float* y, void* y16, int64_t rows, int32_t cols, float scale,
                                   void* stream) {
  MDEMI_REQUIRE(x && y && rows > 0 && cols > 0, "softmax_fwd: bad args");
  return softmax_fwd_launch(x, y, y16, rows, cols, scale, SmDrop{nullptr, 0, 0, 0.f, 1.f}, (hipStream_t)stream);
}

extern "C" int mdemi_softmax_fwd_drop16(const float* x, float* y, void* y16, int64_t rows, int32_t cols, float scale,
                                        float p, const uint64_t* seed_dev, uint64_t seed_add, uint64_t offset,
                                        void* stream) {
  MDEMI_REQUIRE(x && y && y16 && rows > 0 && cols > 0 && p > 0.f && p < 1.f && seed_dev,
                "softmax_fwd_drop16: bad args");
  return softmax_fwd_launch(x, y, y16, rows, cols, scale, SmDrop{seed_dev, seed_add, offset, p, 1.f / (1.f - p)},
                            (hipStream_t)stream);
}

extern "C" int mdemi_softmax_bwd(const float* y, const float* dy, float* dx, int64_t rows, int32_t cols, float scale,
                                 int32_t accumulate, void* stream) {
  return mdemi_softmax_bwd16(y, dy, dx, nullptr, rows, cols, scale, accumulate, stream);
}

extern "C" int mdemi_softmax_bwd16(const float* y, const float* dy, float* dx, void* dx16, int64_t rows, int32_t cols,
                                   float scale, int32_t accumulate, void* stream) {
  MDEMI_REQUIRE(y && dy && dx && rows > 0 && cols > 0, "softmax_bwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  if (cols <= 64 * SM_REG)
    hipLaunchKernelGGL(softmax_wave_bwd, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, st, y, dy, dx, rows, cols, scale,
                       accumulate, (__bf16*)dx16);
  else
    hipLaunchKernelGGL(softmax_block_bwd, dim3((unsigned)rows), dim3(256), 0, st, y, dy, dx, cols, scale, accumulate,
                       (__bf16*)dx16);
  return check_launch("softmax_bwd");
}

extern "C" int mdemi_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed, uint64_t offset,
                             void* stream) {
  MDEMI_REQUIRE(x && y && n > 0 && p >= 0.f && p < 1.f, "dropout: bad args");
  hipStream_t st = (hipStream_t)stream;
  if (p == 0.f) {
    if (x != y) {
      hipError_t e = hipMemcpyAsync(y, x, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, st);
      if (e != hipSuccess) { set_error("dropout: copy failed: %s", hipGetErrorString(e)); return MDEMI_ELAUNCH; }
    }
    return MDEMI_OK;
  }
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_1d(n)), dim3(256), 0, st, x, y, n, p, 1.f / (1.f - p), seed, offset);
  return check_launch("dropout");
}

extern "C" int mdemi_dropout_dev(const float* x, float* y, int64_t n, float p, const uint64_t* seed_dev,
                                 uint64_t seed_add, uint64_t offset, void* stream) {
  return mdemi_dropout_dev16(x, y, nullptr, n, p, seed_dev, seed_add, offset, stream);
}

extern "C" int mdemi_dropout_dev16(const float* x, float* y, void* y16, int64_t n, float p, const uint64_t* seed_dev,
                                   uint64_t seed_add, uint64_t offset, void* stream) {
  MDEMI_REQUIRE(x && y && n > 0 && p > 0.f && p < 1.f && seed_dev, "dropout_dev: bad args");
  const bool v4 = n % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)y16 & 7) == 0;
  MDEMI_REQUIRE(!y16 || v4, "dropout_dev16: the bf16 copy needs n %% 4 == 0 and aligned buffers");
  if (v4) {
    const int64_t n4 = n / 4;
    const unsigned g = (unsigned)std::min<int64_t>(cdiv(n4, 256), 8192);
    hipLaunchKernelGGL(dropout_dev4_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, (const float4*)x, (float4*)y,
                       n4, p, 1.f / (1.f - p), seed_dev, seed_add, offset, (dp_bf16x4_t*)y16);
  } else {
    hipLaunchKernelGGL(dropout_dev_kernel, dim3(grid_1d(n)), dim3(256), 0, (hipStream_t)stream, x, y, n, p,
                       1.f / (1.f - p), seed_dev, seed_add, offset);
  }
  return check_launch("dropout_dev");
}

extern "C" int mdemi_act_fwd(const float* x, float* y, int64_t n, int32_t act, void* stream) {
  MDEMI_REQUIRE(x && y && n > 0, "act_fwd: bad args");
  hipLaunchKernelGGL(act_fwd_kernel, dim3(grid_1d(n)), dim3(256), 0, (hipStream_t)stream, x, y, n, act);
  return check_launch("act_fwd");
}

extern "C" int mdemi_binhead_nhwc_fwd(const float* logits, const float* centers, float* pred, float* stats, int32_t B,
                                      int64_t HW, int32_t K, void* stream) {
  MDEMI_REQUIRE(logits && centers && pred && stats && B > 0 && HW > 0 && K > 0 && K % 4 == 0,
                "binhead_nhwc_fwd: bad args (K %% 4 == 0)");
  const int64_t npix = (int64_t)B * HW;
  hipStream_t st = (hipStream_t)stream;
  const bool al = ((uintptr_t)logits & 15) == 0 && ((uintptr_t)centers & 15) == 0 && ((uintptr_t)stats & 7) == 0;
  if (al && (K == 64 || K == 128 || K == 256 || K == 512)) {
    const unsigned nb = (unsigned)std::min<int64_t>(cdiv(npix, 16), 16384);
    auto k = K == 64 ? binhead_nhwc_fwd_g16<1> : K == 128 ? binhead_nhwc_fwd_g16<2>
           : K == 256 ? binhead_nhwc_fwd_g16<4> : binhead_nhwc_fwd_g16<8>;
    hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, st, logits, centers, pred, stats, HW, npix);
  } else {
    hipLaunchKernelGGL(binhead_nhwc_fwd_kernel, dim3(grid_1d(npix, 4)), dim3(256), 0, st, logits, centers, pred,
                       stats, HW, K, npix);
  }
  return check_launch("binhead_nhwc_fwd");
}

extern "C" size_t mdemi_binhead_nhwc_bwd_workspace_size(int32_t B, int64_t HW, int32_t K) {
  const int64_t nchunk = cdiv(HW, 4 * BH_PIX);
  return align_up((size_t)B * nchunk * K * sizeof(float), 256);
}

extern "C" int mdemi_binhead_nhwc_bwd(const float* logits, const float* centers, const float* pred,
                                      const float* stats, const float* dpred, float* dlogits, float* dcenters,
                                      int32_t B, int64_t HW, int32_t K, void* workspace, void* stream) {
  MDEMI_REQUIRE(logits && centers && pred && stats && dpred && dlogits && dcenters && B > 0 && HW > 0 && K > 0 &&
                    K % 4 == 0 && K <= 4096, "binhead_nhwc_bwd: bad args");
  if (!workspace) { set_error("binhead_nhwc_bwd: workspace required"); return MDEMI_EWORKSPACE; }
  const int nchunk = (int)cdiv(HW, 4 * BH_PIX);
  hipStream_t st = (hipStream_t)stream;
  const bool al = ((uintptr_t)logits & 15) == 0 && ((uintptr_t)centers & 15) == 0 && ((uintptr_t)dlogits & 15) == 0 &&
                  ((uintptr_t)stats & 7) == 0;
  if (al && (K == 64 || K == 128 || K == 256 || K == 512)) {
    auto k = K == 64 ? binhead_nhwc_bwd_g16<1> : K == 128 ? binhead_nhwc_bwd_g16<2>
           : K == 256 ? binhead_nhwc_bwd_g16<4> : binhead_nhwc_bwd_g16<8>;
    hipLaunchKernelGGL(k, dim3(nchunk, B), dim3(256), 0, st, logits, centers, pred, stats, dpred, dlogits,
                       (float*)workspace, HW, nchunk);
  } else {
    hipLaunchKernelGGL(binhead_nhwc_bwd_kernel, dim3(nchunk, B), dim3(256), 4 * K * sizeof(float), st, logits,
                       centers, pred, stats, dpred, dlogits, (float*)workspace, HW, K, nchunk);
  }
  hipLaunchKernelGGL(binhead_nhwc_final, dim3((unsigned)cdiv(K, 64), B), dim3(256), 0, st, (const float*)workspace,
                     dcenters, B, K, nchunk);
  return check_launch("binhead_nhwc_bwd");
}

extern "C" int mdemi_bins_fwd(const float* raw, float* widths_n, float* edges, float* centers, int32_t B, int32_t K,
                              int32_t mode, float min_val, float max_val, void* stream) {
  MDEMI_REQUIRE(raw && centers && B > 0 && K > 0 && (mode == MDEMI_BINS_RELU || mode == MDEMI_BINS_ELU),
                "bins_fwd: bad args");
  hipLaunchKernelGGL(bins_fwd_kernel, dim3((unsigned)cdiv(B, 64)), dim3(64), 0, (hipStream_t)stream, raw, widths_n,
                     edges, centers, B, K, mode, min_val, max_val);
  return check_launch("bins_fwd");
}

extern "C" int mdemi_bins_bwd(const float* raw, const float* dcenters, const float* dedges, const float* dwidths_n,
                              float* draw, int32_t B, int32_t K, int32_t mode, float min_val, float max_val,
                              void* stream) {
  MDEMI_REQUIRE(raw && dcenters && draw && B > 0 && K > 0 && (mode == MDEMI_BINS_RELU || mode == MDEMI_BINS_ELU),
                "bins_bwd: bad args");
  hipLaunchKernelGGL(bins_bwd_kernel, dim3((unsigned)cdiv(B, 64)), dim3(64), 0, (hipStream_t)stream, raw, dcenters,
                     dedges, dwidths_n, draw, B, K, mode, min_val, max_val);
  return check_launch("bins_bwd");
}

extern "C" int mdemi_unpatchify_nhwc(const float* cols, float* x, int32_t N, int32_t H, int32_t W, int32_t C,
                                     int32_t p, int32_t OH, int32_t OW, void* stream) {
  MDEMI_REQUIRE(cols && x && N > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0 && p > 0 && OH * p <= H && OW * p <= W,
                "unpatchify_nhwc: bad args (C %% 4 == 0)");
  const int64_t total = (int64_t)N * H * W * (C / 4);
  hipLaunchKernelGGL(unpatchify_kernel, dim3(grid_1d(total)), dim3(256), 0, (hipStream_t)stream, cols, x, N, H, W, C, p,
                     OH, OW);
  return check_launch("unpatchify_nhwc");
}

extern "C" int mdemi_pad_fold_replicate(const float* dxp, float* dx, int32_t N, int32_t H, int32_t W, int32_t C,
                                        int32_t p, void* stream) {
  MDEMI_REQUIRE(dxp && dx && N > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0 && p >= 0,
                "pad_fold_replicate: bad args (C %% 4 == 0)");
  const int64_t total = (int64_t)N * H * W * (C / 4);
  hipLaunchKernelGGL(pad_fold_kernel, dim3(grid_1d(total)), dim3(256), 0, (hipStream_t)stream, dxp, dx, N, H, W, C,
                     p);
  return check_launch("pad_fold_replicate");
}

extern "C" size_t mdemi_depth_metrics_workspace_size(int32_t B, int32_t H, int32_t W) {
  return align_up((size_t)B * metrics_chunks((int64_t)H * W) * MET_N * sizeof(double), 256);
}

extern "C" int mdemi_depth_metrics(const float* pred, const float* gt, int32_t B, int32_t H, int32_t W, int32_t y0,
                                   int32_t y1, int32_t x0, int32_t x1, float min_depth, float max_depth,
                                   int32_t clamp_pred, double* out, void* workspace, void* stream) {
  MDEMI_REQUIRE(pred && gt && out && B > 0 && H > 0 && W > 0, "depth_metrics: bad args");
  if (!workspace) { set_error("depth_metrics: workspace required"); return MDEMI_EWORKSPACE; }
  const int nchunk = metrics_chunks((int64_t)H * W);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(metrics_partial, dim3(nchunk, B), dim3(256), 0, st, pred, gt, (double*)workspace, H, W, y0, y1,
                     x0, x1, min_depth, max_depth, clamp_pred, nchunk);
  hipLaunchKernelGGL(metrics_final, dim3((unsigned)cdiv(B, 64)), dim3(64), 0, st, (const double*)workspace, out, B,
                     nchunk);
  return check_launch("depth_metrics");
}
