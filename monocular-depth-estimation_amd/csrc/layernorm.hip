// LayerNorm over the last dimension of token-major rows (nn.LayerNorm):
// swin_transformer.py:176,182,260,416,541; newcrf_layers.py:182,188,413;
// luna_layer.py:153-155; feed_forward.py:21; self_attention.py:23.
// One wave per row; the row is cached in registers (CACHE float4 per lane) so
// HBM sees one read and one write per element; statistics are two-pass
// (mean, then centred sum of squares) like ATen's reference semantics.
#include "common.h"

namespace mdemi {

constexpr int LN_THREADS = 256;

typedef __bf16 ln_bf16x4_t __attribute__((ext_vector_type(4)));
typedef float ln_f32x4_t __attribute__((ext_vector_type(4)));

// y16 (optional): the RNE bf16 copy of y, for a bf16 GEMM that reads the output (bf16 storage)
template <int CACHE>
__global__ __launch_bounds__(LN_THREADS) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                           const float* __restrict__ bta, float* __restrict__ y,
                                                           float* __restrict__ mean, float* __restrict__ rstd,
                                                           int64_t rows, int C, float eps,
                                                           __bf16* __restrict__ y16) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * LN_THREADS + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * LN_THREADS) >> 6;
  const int C4 = C >> 2;
  for (int64_t r = wave; r < rows; r += nwaves) {
    const float4* xr = reinterpret_cast<const float4*>(x + r * C);
    float4 v[CACHE];
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < CACHE; ++q) {
      const int c4 = lane + 64 * q;
      v[q] = c4 < C4 ? xr[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
      s += (v[q].x + v[q].y) + (v[q].z + v[q].w);
    }
    const float mu = wave_sum(s) / (float)C;
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < CACHE; ++q) {
      const int c4 = lane + 64 * q;
      if (c4 < C4) {
        const float a = v[q].x - mu, b = v[q].y - mu, c = v[q].z - mu, d = v[q].w - mu;
        ss += (a * a + b * b) + (c * c + d * d);
      }
    }
    const float rs = rsqrtf(wave_sum(ss) / (float)C + eps);
    float4* yr = reinterpret_cast<float4*>(y + r * C);
#pragma unroll
    for (int q = 0; q < CACHE; ++q) {
      const int c4 = lane + 64 * q;
      if (c4 < C4) {
        const float4 gg = reinterpret_cast<const float4*>(g)[c4];
        const float4 bb = reinterpret_cast<const float4*>(bta)[c4];
        float4 o;
        o.x = (v[q].x - mu) * rs * gg.x + bb.x;
        o.y = (v[q].y - mu) * rs * gg.y + bb.y;
        o.z = (v[q].z - mu) * rs * gg.z + bb.z;
        o.w = (v[q].w - mu) * rs * gg.w + bb.w;
        yr[c4] = o;
        if (y16) {
          const ln_f32x4_t ov = {o.x, o.y, o.z, o.w};
          *reinterpret_cast<ln_bf16x4_t*>(y16 + r * C + 4 * c4) = __builtin_convertvector(ov, ln_bf16x4_t);
        }
      }
    }
    if (lane == 0) {
      if (mean) mean[r] = mu;
      if (rstd) rstd[r] = rs;
    }
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat))
// dgamma/dbeta: per-lane register partials over the rows a block visits, then
// one [2][C] partial row per block in the workspace (reduced deterministically).
template <int CACHE>
__global__ __launch_bounds__(LN_THREADS) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                           const float* __restrict__ mean, const float* __restrict__ rstd,
                                                           const float* __restrict__ g, float* dx,
                                                           float* __restrict__ partial, int64_t rows, int C,
                                                           const float* addsrc) {
  __shared__ float4 red[LN_THREADS / 64][128];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * LN_THREADS + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * LN_THREADS) >> 6;
  const int C4 = C >> 2;
  float4 dg[CACHE], db[CACHE], gg[CACHE];
#pragma unroll
  for (int q = 0; q < CACHE; ++q) {
    dg[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    db[q] = dg[q];
    const int c4 = lane + 64 * q;
    gg[q] = c4 < C4 ? reinterpret_cast<const float4*>(g)[c4] : dg[q];
  }
  for (int64_t r = wave; r < rows; r += nwaves) {
    const float mu = mean[r], rs = rstd[r];
    const float4* xr = reinterpret_cast<const float4*>(x + r * C);
    const float4* dyr = reinterpret_cast<const float4*>(dy + r * C);
    float4 xh[CACHE], gd[CACHE];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < CACHE; ++q) {
      const int c4 = lane + 64 * q;
      if (c4 < C4) {
        const float4 xv = xr[c4], d = dyr[c4];
        xh[q] = make_float4((xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs);
        gd[q] = make_float4(d.x * gg[q].x, d.y * gg[q].y, d.z * gg[q].z, d.w * gg[q].w);
        s1 += (gd[q].x + gd[q].y) + (gd[q].z + gd[q].w);
        s2 += (gd[q].x * xh[q].x + gd[q].y * xh[q].y) + (gd[q].z * xh[q].z + gd[q].w * xh[q].w);
        dg[q].x += d.x * xh[q].x; dg[q].y += d.y * xh[q].y; dg[q].z += d.z * xh[q].z; dg[q].w += d.w * xh[q].w;
        db[q].x += d.x; db[q].y += d.y; db[q].z += d.z; db[q].w += d.w;
      } else {
        xh[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        gd[q] = xh[q];
      }
    }
    const float m1 = wave_sum(s1) / (float)C, m2 = wave_sum(s2) / (float)C;
    float4* dxr = reinterpret_cast<float4*>(dx + r * C);
#pragma unroll
    for (int q = 0; q < CACHE; ++q) {
      const int c4 = lane + 64 * q;
      if (c4 < C4) {
        float4 o;
        o.x = rs * (gd[q].x - m1 - xh[q].x * m2);
        o.y = rs * (gd[q].y - m1 - xh[q].y * m2);
        o.z = rs * (gd[q].z - m1 - xh[q].z * m2);
        o.w = rs * (gd[q].w - m1 - xh[q].w * m2);
        if (addsrc) {  // dx = LN'(dy) + addsrc (addsrc may be dx itself)
          const float4 p = reinterpret_cast<const float4*>(addsrc + r * C)[c4];
          o.x += p.x; o.y += p.y; o.z += p.z; o.w += p.w;
        }
        dxr[c4] = o;
      }
    }
  }
  float* P = partial + (int64_t)blockIdx.x * 2 * C;
#pragma unroll
  for (int q = 0; q < CACHE; ++q) {
    red[wid][lane] = dg[q];
    red[wid][64 + lane] = db[q];
    __syncthreads();
    if (threadIdx.x < 128) {
      const int which = threadIdx.x >> 6, ln = threadIdx.x & 63;
      const int c4 = ln + 64 * q;
      if (c4 < C4) {
        float4 s = red[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < LN_THREADS / 64; ++w) {
          const float4 t = red[w][threadIdx.x];
          s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
        }
        *reinterpret_cast<float4*>(P + which * C + 4 * c4) = s;
      }
    }
    __syncthreads();
  }
}

__global__ void ln_param_split(const float* __restrict__ sums, float* __restrict__ dgamma, float* __restrict__ dbeta,
                               int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dgamma) dgamma[c] = sums[c];
  if (dbeta) dbeta[c] = sums[C + c];
}

static int ln_cache(int C) {
  const int c4 = (C + 3) / 4;
  if (c4 <= 64) return 1;
  if (c4 <= 128) return 2;
  if (c4 <= 256) return 4;
  if (c4 <= 512) return 8;
  if (c4 <= 1536) return 24;
  return -1;
}
static int ln_fwd_blocks(int64_t rows) {
  const int64_t nb = cdiv(rows, LN_THREADS / 64);
  return (int)(nb < 8192 ? nb : 8192);
}
static int ln_bwd_blocks(int64_t rows, int C) {
  // keep the [blocks][2][C] partial buffer modest
  int cap = C <= 512 ? 1024 : 512;
  const int64_t nb = cdiv(rows, LN_THREADS / 64);
  return (int)(nb < cap ? nb : cap);
}

}  // namespace mdemi

using namespace mdemi;

#define LN_DISPATCH(CACHEV, KERNEL, ...)                                          \
  switch (CACHEV) {                                                               \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                    \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                    \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                    \
    case 8: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break;                    \
    default: hipLaunchKernelGGL(KERNEL<24>, __VA_ARGS__); break;                  \
  }

extern "C" int mdemi_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y,
                                   float* mean, float* rstd, int64_t rows, int32_t C, float eps,
                                   void* stream) {
  return mdemi_layernorm_fwd16(x, gamma, beta, y, nullptr, mean, rstd, rows, C, eps, stream);
}

extern "C" int mdemi_layernorm_fwd16(const float* x, const float* gamma, const float* beta, float* y, void* y16,
                                     float* mean, float* rstd, int64_t rows, int32_t C, float eps, void* stream) {
  MDEMI_REQUIRE(x && gamma && beta && y && rows > 0 && C > 0, "layernorm_fwd: bad args");
  MDEMI_REQUIRE(!y16 || ((uintptr_t)y16 & 7) == 0, "layernorm_fwd16: y16 must be 8-B aligned");
  MDEMI_REQUIRE(C % 4 == 0, "layernorm_fwd: C %% 4 != 0 (C=%d)", C);
  const int cache = ln_cache(C);
  MDEMI_REQUIRE(cache > 0, "layernorm_fwd: C=%d too large", C);
  hipStream_t st = (hipStream_t)stream;
  LN_DISPATCH(cache, ln_fwd_kernel, dim3(ln_fwd_blocks(rows)), dim3(LN_THREADS), 0, st, x, gamma, beta, y, mean,
              rstd, rows, C, eps, (__bf16*)y16);
  return check_launch("layernorm_fwd");
}

// workspace: [partials nb x 2C | sums 2C | colsum scratch]
static size_t ln_part_bytes(int64_t rows, int C) { return align_up((size_t)ln_bwd_blocks(rows, C) * 2 * C * 4, 256); }
extern "C" size_t mdemi_layernorm_bwd_workspace_size(int64_t rows, int32_t C) {
  return ln_part_bytes(rows, C) + align_up((size_t)2 * C * 4, 256) + colsum_ws_bytes(ln_bwd_blocks(rows, C), 2 * C);
}

static int ln_bwd_launch(const float* dy, const float* x, const float* mean, const float* rstd, const float* gamma,
                         const float* addsrc, float* dx, float* dgamma, float* dbeta, int64_t rows, int32_t C,
                         void* workspace, hipStream_t st) {
  MDEMI_REQUIRE(dy && x && mean && rstd && gamma && dx && rows > 0 && C > 0, "layernorm_bwd: bad args");
  MDEMI_REQUIRE(C % 4 == 0, "layernorm_bwd: C %% 4 != 0 (C=%d)", C);
  const int cache = ln_cache(C);
  MDEMI_REQUIRE(cache > 0, "layernorm_bwd: C=%d too large", C);
  if (!workspace) { set_error("layernorm_bwd: workspace required"); return MDEMI_EWORKSPACE; }
  const int nb = ln_bwd_blocks(rows, C);
  float* partial = (float*)workspace;
  LN_DISPATCH(cache, ln_bwd_kernel, dim3(nb), dim3(LN_THREADS), 0, st, dy, x, mean, rstd, gamma, dx, partial, rows,
              C, addsrc);
  if (dgamma || dbeta) {
    float* sums = (float*)((char*)workspace + ln_part_bytes(rows, C));
    void* cws = (char*)sums + align_up((size_t)2 * C * 4, 256);
    if (dgamma && dbeta)  // the partial sums land in dgamma / dbeta directly
      return colsum_launch_split(partial, nb, 2 * C, 2 * C, dgamma, dbeta, C, 0, cws, st);
    int rc = colsum_launch(partial, nb, 2 * C, 2 * C, sums, 0, cws, st);
    if (rc) return rc;
    hipLaunchKernelGGL(ln_param_split, dim3((C + 255) / 256), dim3(256), 0, st, sums, dgamma, dbeta, C);
  }
  return check_launch("layernorm_bwd");
}

extern "C" int mdemi_layernorm_bwd(const float* dy, const float* x, const float* mean, const float* rstd,
                                   const float* gamma, float* dx, float* dgamma, float* dbeta, int64_t rows,
                                   int32_t C, int32_t accumulate_dx, void* workspace, void* stream) {
  return ln_bwd_launch(dy, x, mean, rstd, gamma, accumulate_dx ? dx : nullptr, dx, dgamma, dbeta, rows, C, workspace,
                       (hipStream_t)stream);
}

extern "C" int mdemi_layernorm_bwd_add(const float* dy, const float* x, const float* mean, const float* rstd,
                                       const float* gamma, const float* dadd, float* dx, float* dgamma, float* dbeta,
                                       int64_t rows, int32_t C, void* workspace, void* stream) {
  MDEMI_REQUIRE(dadd, "layernorm_bwd_add: dadd required");
  return ln_bwd_launch(dy, x, mean, rstd, gamma, dadd, dx, dgamma, dbeta, rows, C, workspace, (hipStream_t)stream);
}
