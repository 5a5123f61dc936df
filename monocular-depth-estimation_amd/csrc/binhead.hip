// Adaptive-bin depth head: per-pixel softmax over K bins + sum_k p_k * c_k.
// Reference: model/Adabins/unet_adaptive_bins.py:88-107 (conv_out softmax,
// pred = sum(out * centers)), model/Depthformer/depthformer_v8.py:62-73 and
// decoder_v8.py:158-159.
//
// Layout [B][K][HW] (the reference's NCHW logits).  One lane owns VEC
// consecutive pixels and sweeps the K bins with an online softmax, so every
// load instruction reads 64*VEC consecutive pixels of one bin (fully
// coalesced) and no cross-lane reduction is needed on the forward.  The
// kernel is HBM-bound: forward reads K*HW*4 B and writes 3*HW*4 B per image.
#include "common.h"

namespace mdemi {

template <int VEC>
struct vecf;
template <>
struct vecf<4> {
  using T = float4;
  __device__ static T load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  __device__ static void store(float* p, T v) { *reinterpret_cast<float4*>(p) = v; }
  __device__ static float get(const T& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
  __device__ static void set(T& v, int i, float x) {
    if (i == 0) v.x = x; else if (i == 1) v.y = x; else if (i == 2) v.z = x; else v.w = x;
  }
};
template <>
struct vecf<1> {
  using T = float;
  __device__ static T load(const float* p) { return *p; }
  __device__ static void store(float* p, T v) { *p = v; }
  __device__ static float get(const T& v, int) { return v; }
  __device__ static void set(T& v, int, float x) { v = x; }
};

constexpr int BH_THREADS = 256;
constexpr int BH_CHUNK = 8;  // bins per max-rescale step

// grid: (pixel-group blocks, B)
template <int VEC>
__global__ __launch_bounds__(BH_THREADS) void binhead_fwd_kernel(
    const float* __restrict__ logits, const float* __restrict__ centers, float* __restrict__ pred,
    float* __restrict__ stats, float* __restrict__ probs, int K, int64_t HW, int do_softmax) {
  using V = vecf<VEC>;
  const int b = blockIdx.y;
  const float* L = logits + (int64_t)b * K * HW;
  const float* Cb = centers + (int64_t)b * K;
  const int64_t ngroups = HW / VEC;
  for (int64_t g = (int64_t)blockIdx.x * BH_THREADS + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * BH_THREADS) {
    const int64_t px = g * VEC;
    float m[VEC], s[VEC], t[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) { m[v] = -INFINITY; s[v] = 0.f; t[v] = 0.f; }
    if (do_softmax) {
      int k0 = 0;
      for (; k0 + BH_CHUNK <= K; k0 += BH_CHUNK) {
        typename V::T x[BH_CHUNK];
#pragma unroll
        for (int j = 0; j < BH_CHUNK; ++j) x[j] = V::load(L + (int64_t)(k0 + j) * HW + px);
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          float cm = m[v];
#pragma unroll
          for (int j = 0; j < BH_CHUNK; ++j) cm = fmaxf(cm, V::get(x[j], v));
          const float a = __expf(m[v] - cm);
          float ss = s[v] * a, tt = t[v] * a;
#pragma unroll
          for (int j = 0; j < BH_CHUNK; ++j) {
            const float e = __expf(V::get(x[j], v) - cm);
            ss += e;
            tt = fmaf(e, Cb[k0 + j], tt);
          }
          m[v] = cm; s[v] = ss; t[v] = tt;
        }
      }
      for (; k0 < K; ++k0) {
        typename V::T x = V::load(L + (int64_t)k0 * HW + px);
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const float xv = V::get(x, v);
          const float cm = fmaxf(m[v], xv);
          const float a = __expf(m[v] - cm), e = __expf(xv - cm);
          s[v] = s[v] * a + e;
          t[v] = fmaf(e, Cb[k0], t[v] * a);
          m[v] = cm;
        }
      }
      typename V::T pv, mv, iv;
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const float inv = 1.f / s[v];
        V::set(pv, v, t[v] * inv);
        V::set(mv, v, m[v]);
        V::set(iv, v, inv);
      }
      V::store(pred + (int64_t)b * HW + px, pv);
      if (stats) {
        V::store(stats + ((int64_t)b * 2 + 0) * HW + px, mv);
        V::store(stats + ((int64_t)b * 2 + 1) * HW + px, iv);
      }
      if (probs) {
        for (int k = 0; k < K; ++k) {
          typename V::T x = V::load(L + (int64_t)k * HW + px), o;
#pragma unroll
          for (int v = 0; v < VEC; ++v) V::set(o, v, __expf(V::get(x, v) - V::get(mv, v)) * V::get(iv, v));
          V::store(probs + ((int64_t)b * K + k) * HW + px, o);
        }
      }
    } else {
      for (int k = 0; k < K; ++k) {
        typename V::T x = V::load(L + (int64_t)k * HW + px);
        const float c = Cb[k];
#pragma unroll
        for (int v = 0; v < VEC; ++v) t[v] = fmaf(V::get(x, v), c, t[v]);
      }
      typename V::T pv;
#pragma unroll
      for (int v = 0; v < VEC; ++v) V::set(pv, v, t[v]);
      V::store(pred + (int64_t)b * HW + px, pv);
    }
  }
}

// Backward.  dlogits_k = p_k * (c_k - pred) * dpred   (softmax head)
//            dprobs_k  = c_k * dpred                   (probabilities given)
// dcenters[b,k] = sum_px p_k * dpred: per-wave partials in LDS, one partial row
// per block in the workspace, reduced by binhead_dcenters_reduce (deterministic).
template <int VEC>
__global__ __launch_bounds__(BH_THREADS) void binhead_bwd_kernel(
    const float* __restrict__ logits, const float* __restrict__ centers,
    const float* __restrict__ pred, const float* __restrict__ stats,
    const float* __restrict__ dpred, float* __restrict__ dlogits, float* __restrict__ partial,
    int K, int64_t HW, int do_softmax) {
  using V = vecf<VEC>;
  extern __shared__ float red[];  // [4 waves][K]
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int k = threadIdx.x; k < 4 * K; k += BH_THREADS) red[k] = 0.f;
  __syncthreads();
  const float* L = logits + (int64_t)b * K * HW;
  float* D = dlogits + (int64_t)b * K * HW;
  const float* Cb = centers + (int64_t)b * K;
  const int64_t ngroups = HW / VEC;
  // every lane of a wave runs the same number of iterations (wave-uniform trip
  // count) so the per-bin wave reduction below sees all 64 lanes.
  const int64_t stride = (int64_t)gridDim.x * BH_THREADS;
  const int64_t g0 = (int64_t)blockIdx.x * BH_THREADS + (threadIdx.x & ~63);
  for (int64_t gb = g0; gb < ngroups; gb += stride) {
    const int64_t g = gb + lane;
    const bool active = g < ngroups;
    const int64_t px = (active ? g : 0) * VEC;
    typename V::T mv, iv, pr, dp;
    if (active) {
      pr = V::load(pred + (int64_t)b * HW + px);
      dp = V::load(dpred + (int64_t)b * HW + px);
      if (do_softmax) {
        mv = V::load(stats + ((int64_t)b * 2 + 0) * HW + px);
        iv = V::load(stats + ((int64_t)b * 2 + 1) * HW + px);
      }
    } else {
#pragma unroll
      for (int v = 0; v < VEC; ++v) { V::set(pr, v, 0.f); V::set(dp, v, 0.f); V::set(mv, v, 0.f); V::set(iv, v, 0.f); }
    }
    for (int k = 0; k < K; ++k) {
      const float c = Cb[k];
      float acc = 0.f;
      if (active) {
        typename V::T x = V::load(L + (int64_t)k * HW + px), o;
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const float d = V::get(dp, v);
          if (do_softmax) {
            const float p = __expf(V::get(x, v) - V::get(mv, v)) * V::get(iv, v);
            V::set(o, v, p * (c - V::get(pr, v)) * d);
            acc = fmaf(p, d, acc);
          } else {
            V::set(o, v, c * d);
            acc = fmaf(V::get(x, v), d, acc);
          }
        }
        V::store(D + (int64_t)k * HW + px, o);
      }
      acc = wave_sum(acc);
      if (lane == 0) red[wid * K + k] += acc;
    }
  }
  __syncthreads();
  float* P = partial + ((int64_t)b * gridDim.x + blockIdx.x) * K;
  for (int k = threadIdx.x; k < K; k += BH_THREADS)
    P[k] = red[k] + red[K + k] + red[2 * K + k] + red[3 * K + k];
}

__global__ void binhead_dcenters_reduce(const float* __restrict__ partial, float* __restrict__ dcenters,
                                        int K, int nblk) {
  const int b = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float s = 0.f;
  for (int i = 0; i < nblk; ++i) s += partial[((int64_t)b * nblk + i) * K + k];
  dcenters[(int64_t)b * K + k] = s;
}

static int bh_blocks(int64_t groups) {
  int64_t nb = cdiv(groups, BH_THREADS);
  return (int)(nb < 1024 ? (nb < 1 ? 1 : nb) : 1024);
}
static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace mdemi

using namespace mdemi;

extern "C" int mdemi_binhead_fwd(const float* logits, const float* centers, float* pred,
                                 float* stats, float* probs_out, int32_t B, int32_t K, int64_t HW,
                                 int32_t do_softmax, void* stream) {
  MDEMI_REQUIRE(logits && centers && pred && B > 0 && K > 0 && HW > 0, "binhead_fwd: bad args");
  MDEMI_REQUIRE(!do_softmax || stats || !probs_out, "binhead_fwd: probs_out requires stats");
  hipStream_t st = (hipStream_t)stream;
  const bool v4 = (HW % 4 == 0) && aligned16(logits) && aligned16(pred) &&
                  (!stats || aligned16(stats)) && (!probs_out || aligned16(probs_out));
  if (v4) {
    dim3 grid(bh_blocks(HW / 4), B);
    hipLaunchKernelGGL(binhead_fwd_kernel<4>, grid, dim3(BH_THREADS), 0, st, logits, centers, pred,
                       stats, probs_out, K, HW, do_softmax);
  } else {
    dim3 grid(bh_blocks(HW), B);
    hipLaunchKernelGGL(binhead_fwd_kernel<1>, grid, dim3(BH_THREADS), 0, st, logits, centers, pred,
                       stats, probs_out, K, HW, do_softmax);
  }
  return check_launch("binhead_fwd");
}

static int bh_bwd_blocks(int64_t HW, bool v4) {
  const int64_t groups = v4 ? HW / 4 : HW;
  int64_t nb = cdiv(groups, BH_THREADS);
  return (int)(nb < 256 ? (nb < 1 ? 1 : nb) : 256);
}

extern "C" size_t mdemi_binhead_bwd_workspace_size(int32_t B, int32_t K, int64_t HW) {
  const int nb = bh_bwd_blocks(HW, false);  // upper bound over both paths
  return (size_t)B * nb * K * sizeof(float);
}

extern "C" int mdemi_binhead_bwd(const float* logits, const float* centers, const float* pred,
                                 const float* stats, const float* dpred, float* dlogits,
                                 float* dcenters, int32_t B, int32_t K, int64_t HW,
                                 int32_t do_softmax, void* workspace, void* stream) {
  MDEMI_REQUIRE(logits && centers && pred && dpred && dlogits && dcenters && B > 0 && K > 0 && HW > 0,
                "binhead_bwd: bad args");
  MDEMI_REQUIRE(!do_softmax || stats, "binhead_bwd: softmax head needs the forward stats");
  if (!workspace) { set_error("binhead_bwd: workspace required"); return MDEMI_EWORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  const bool v4 = (HW % 4 == 0) && aligned16(logits) && aligned16(pred) && aligned16(dpred) &&
                  aligned16(dlogits) && (!stats || aligned16(stats));
  const int nb = bh_bwd_blocks(HW, v4);
  const size_t lds = 4 * (size_t)K * sizeof(float);
  MDEMI_REQUIRE(lds <= 64 * 1024, "binhead_bwd: K=%d too large", K);
  float* partial = (float*)workspace;
  dim3 grid(nb, B);
  if (v4)
    hipLaunchKernelGGL(binhead_bwd_kernel<4>, grid, dim3(BH_THREADS), lds, st, logits, centers, pred,
                       stats, dpred, dlogits, partial, K, HW, do_softmax);
  else
    hipLaunchKernelGGL(binhead_bwd_kernel<1>, grid, dim3(BH_THREADS), lds, st, logits, centers, pred,
                       stats, dpred, dlogits, partial, K, HW, do_softmax);
  dim3 g2((K + 255) / 256, B);
  hipLaunchKernelGGL(binhead_dcenters_reduce, g2, dim3(256), 0, st, partial, dcenters, K, nb);
  return check_launch("binhead_bwd");
}
