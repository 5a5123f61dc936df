// Training-mode channel normalisation over NHWC activations with a fused
// activation: BatchNorm2d (statistics per channel over N*H*W;
// uper_crf_head.py:341-348 through mmcv ConvModule, unet_adaptive_bins.py:13,16,
// layer_utils.py:25) and GroupNorm (statistics per (n, group) over H*W*C/G;
// uper_crf_head.py:35 — the PPM's num_groups=256 override).
// Variance is the biased batch variance used for normalisation (ATen
// semantics); the unbiased value for running_var is derived by the caller.
#include "common.h"

namespace mdemi {

constexpr int CN_THREADS = 256;

// ---- BatchNorm statistics: per-block partial [blk][C] of sum (pass 0) or
// centred sum of squares (pass 1, given mean) ----
__global__ __launch_bounds__(CN_THREADS) void bn_partial(const float* __restrict__ x, const float* __restrict__ mean,
                                                         float* __restrict__ part, int64_t rows, int C, int pass,
                                                         int rows_per_blk) {
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = min(rows, r0 + rows_per_blk);
  for (int c = threadIdx.x; c < C; c += CN_THREADS) {
    const float mu = pass ? mean[c] : 0.f;
    float s = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
      const float v = x[r * C + c] - mu;
      s = pass ? fmaf(v, v, s) : s + v;
    }
    part[(int64_t)blockIdx.x * C + c] = s;
  }
}

__global__ void bn_combine(const float* __restrict__ part, int nblk, int C, int64_t rows, int pass, float eps,
                           float* __restrict__ mean, float* __restrict__ rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int i = 0; i < nblk; ++i) s += part[(int64_t)i * C + c];
  if (pass == 0) mean[c] = (float)(s / (double)rows);
  else rstd[c] = (float)(1.0 / sqrt(s / (double)rows + (double)eps));
}

// ---- GroupNorm statistics: one block per (n, group) ----
__global__ __launch_bounds__(CN_THREADS) void gn_stats(const float* __restrict__ x, float* __restrict__ mean,
                                                       float* __restrict__ rstd, int64_t HW, int C, int G, float eps) {
  __shared__ float red[CN_THREADS / 64];
  const int n = blockIdx.x / G, g = blockIdx.x % G;
  const int cpg = C / G;
  const int64_t cnt = HW * cpg;
  const float* X = x + (int64_t)n * HW * C + g * cpg;
  float s = 0.f;
  for (int64_t e = threadIdx.x; e < cnt; e += CN_THREADS) s += X[(e / cpg) * C + e % cpg];
  const float mu = block_sum<CN_THREADS>(s, red) / (float)cnt;
  float ss = 0.f;
  for (int64_t e = threadIdx.x; e < cnt; e += CN_THREADS) {
    const float v = X[(e / cpg) * C + e % cpg] - mu;
    ss = fmaf(v, v, ss);
  }
  const float var = block_sum<CN_THREADS>(ss, red) / (float)cnt;
  if (threadIdx.x == 0) {
    mean[blockIdx.x] = mu;
    rstd[blockIdx.x] = rsqrtf(var + eps);
  }
}

// y = act((x - mean) * rstd * gamma + beta); stat index = channel (BN) or n*G + c/cpg (GN)
__global__ __launch_bounds__(CN_THREADS) void chnorm_apply(const float* __restrict__ x, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, float* __restrict__ y,
                                                           int N, int64_t HW, int C, int G, int is_bn, int act) {
  const int64_t total = (int64_t)N * HW * C;
  const int cpg = C / G;
  for (int64_t e = (int64_t)blockIdx.x * CN_THREADS + threadIdx.x; e < total; e += (int64_t)gridDim.x * CN_THREADS) {
    const int c = (int)(e % C);
    const int s = is_bn ? c : (int)(e / (HW * C)) * G + c / cpg;
    const float v = (x[e] - mean[s]) * rstd[s] * gamma[c] + beta[c];
    y[e] = apply_act(act, v);
  }
}

// ---- backward ----
// pass A: per-block partial [blk][2][C] of (sum dpre*xhat, sum dpre) (BN: over rows;
// GN: handled per (n,group) below).  dpre = dy * act'(pre), pre recomputed.
__global__ __launch_bounds__(CN_THREADS) void bn_bwd_partial(const float* __restrict__ dy, const float* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float* __restrict__ part,
                                                             int64_t rows, int C, int act, int rows_per_blk) {
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = min(rows, r0 + rows_per_blk);
  for (int c = threadIdx.x; c < C; c += CN_THREADS) {
    const float mu = mean[c], rs = rstd[c], ga = gamma[c], be = beta[c];
    float sdx = 0.f, sd = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
      const float xh = (x[r * C + c] - mu) * rs;
      const float pre = xh * ga + be;
      const float d = dy[r * C + c] * act_grad(act, pre, apply_act(act, pre));
      sdx = fmaf(d, xh, sdx);
      sd += d;
    }
    part[((int64_t)blockIdx.x * 2 + 0) * C + c] = sdx;
    part[((int64_t)blockIdx.x * 2 + 1) * C + c] = sd;
  }
}

__global__ void bn_bwd_combine(const float* __restrict__ part, int nblk, int C, float* __restrict__ dgamma,
                               float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  // fp64 combine, as for the forward statistics: dx subtracts these means
  // from d, so their rounding is what survives the cancellation
  double a = 0.0, b = 0.0;
  for (int i = 0; i < nblk; ++i) {
    a += (double)part[((int64_t)i * 2 + 0) * C + c];
    b += (double)part[((int64_t)i * 2 + 1) * C + c];
  }
  dgamma[c] = (float)a;
  dbeta[c] = (float)b;
}

__global__ __launch_bounds__(CN_THREADS) void bn_bwd_apply(const float* __restrict__ dy, const float* __restrict__ x,
                                                           const float* __restrict__ mean, const float* __restrict__ rstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ dgamma,
                                                           const float* __restrict__ dbeta, float* __restrict__ dx,
                                                           int64_t rows, int C, int act) {
  const int64_t total = rows * C;
  const float inv_n = 1.f / (float)rows;
  for (int64_t e = (int64_t)blockIdx.x * CN_THREADS + threadIdx.x; e < total; e += (int64_t)gridDim.x * CN_THREADS) {
    const int c = (int)(e % C);
    const float rs = rstd[c], ga = gamma[c];
    const float xh = (x[e] - mean[c]) * rs;
    const float pre = xh * ga + beta[c];
    const float d = dy[e] * act_grad(act, pre, apply_act(act, pre));
    dx[e] = ga * rs * (d - inv_n * dbeta[c] - xh * inv_n * dgamma[c]);
  }
}

// GroupNorm backward: one block per (n, group); also writes per-(n) partial
// parameter gradients part[n][2][C] reduced over n afterwards.
__global__ __launch_bounds__(CN_THREADS) void gn_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float* __restrict__ dx,
                                                            float* __restrict__ part, int64_t HW, int C, int G,
                                                            int act) {
  __shared__ float red[CN_THREADS / 64];
  const int n = blockIdx.x / G, g = blockIdx.x % G;
  const int cpg = C / G;
  const int64_t cnt = HW * cpg;
  const float mu = mean[blockIdx.x], rs = rstd[blockIdx.x];
  const int64_t base = (int64_t)n * HW * C + g * cpg;
  float s1 = 0.f, s2 = 0.f;
  for (int64_t e = threadIdx.x; e < cnt; e += CN_THREADS) {
    const int c = g * cpg + (int)(e % cpg);
    const int64_t off = base + (e / cpg) * C + e % cpg;
    const float xh = (x[off] - mu) * rs;
    const float pre = xh * gamma[c] + beta[c];
    const float gd = dy[off] * act_grad(act, pre, apply_act(act, pre)) * gamma[c];
    s1 += gd;
    s2 = fmaf(gd, xh, s2);
  }
  const float m1 = block_sum<CN_THREADS>(s1, red) / (float)cnt;
  const float m2 = block_sum<CN_THREADS>(s2, red) / (float)cnt;
  for (int64_t e = threadIdx.x; e < cnt; e += CN_THREADS) {
    const int c = g * cpg + (int)(e % cpg);
    const int64_t off = base + (e / cpg) * C + e % cpg;
    const float xh = (x[off] - mu) * rs;
    const float pre = xh * gamma[c] + beta[c];
    const float gd = dy[off] * act_grad(act, pre, apply_act(act, pre)) * gamma[c];
    dx[off] = rs * (gd - m1 - xh * m2);
  }
  // parameter-gradient partials for this (n, group): channels of the group
  for (int cl = threadIdx.x; cl < cpg; cl += CN_THREADS) {
    const int c = g * cpg + cl;
    float a = 0.f, b = 0.f;
    for (int64_t r = 0; r < HW; ++r) {
      const int64_t off = (int64_t)n * HW * C + r * C + c;
      const float xh = (x[off] - mu) * rs;
      const float pre = xh * gamma[c] + beta[c];
      const float d = dy[off] * act_grad(act, pre, apply_act(act, pre));
      a = fmaf(d, xh, a);
      b += d;
    }
    part[((int64_t)n * 2 + 0) * C + c] = a;
    part[((int64_t)n * 2 + 1) * C + c] = b;
  }
}

static int rows_per_block(int64_t rows) {
  // ~256 partial blocks
  int64_t rpb = cdiv(rows, 256);
  return (int)(rpb < 1 ? 1 : rpb);
}
static int grid_for(int64_t total) {
  const int64_t nb = cdiv(total, CN_THREADS);
  return (int)(nb < 8192 ? (nb < 1 ? 1 : nb) : 8192);
}

}  // namespace mdemi

using namespace mdemi;

extern "C" size_t mdemi_chnorm_workspace_size(int32_t N, int64_t HW, int32_t C, int32_t groups, int32_t is_bn) {
  (void)groups;
  if (is_bn) {
    const int64_t rows = (int64_t)N * HW;
    const int64_t nblk = cdiv(rows, rows_per_block(rows));
    return (size_t)nblk * 2 * C * sizeof(float);
  }
  return (size_t)N * 2 * C * sizeof(float);
}

extern "C" int mdemi_chnorm_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean,
                                float* rstd, int32_t N, int64_t HW, int32_t C, int32_t groups, int32_t is_bn, float eps,
                                int32_t act, void* workspace, void* stream) {
  MDEMI_REQUIRE(x && gamma && beta && y && mean && rstd && N > 0 && HW > 0 && C > 0, "chnorm_fwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  if (is_bn) {
    if (!workspace) { set_error("chnorm_fwd: workspace required"); return MDEMI_EWORKSPACE; }
    const int64_t rows = (int64_t)N * HW;
    const int rpb = rows_per_block(rows);
    const int nblk = (int)cdiv(rows, rpb);
    float* part = (float*)workspace;
    hipLaunchKernelGGL(bn_partial, dim3(nblk), dim3(CN_THREADS), 0, st, x, mean, part, rows, C, 0, rpb);
    hipLaunchKernelGGL(bn_combine, dim3((C + 255) / 256), dim3(256), 0, st, part, nblk, C, rows, 0, eps, mean, rstd);
    hipLaunchKernelGGL(bn_partial, dim3(nblk), dim3(CN_THREADS), 0, st, x, mean, part, rows, C, 1, rpb);
    hipLaunchKernelGGL(bn_combine, dim3((C + 255) / 256), dim3(256), 0, st, part, nblk, C, rows, 1, eps, mean, rstd);
    hipLaunchKernelGGL(chnorm_apply, dim3(grid_for(rows * C)), dim3(CN_THREADS), 0, st, x, gamma, beta, mean, rstd, y,
                       N, HW, C, C, 1, act);
  } else {
    MDEMI_REQUIRE(groups > 0 && C % groups == 0, "chnorm_fwd: C %% groups != 0");
    hipLaunchKernelGGL(gn_stats, dim3(N * groups), dim3(CN_THREADS), 0, st, x, mean, rstd, HW, C, groups, eps);
    hipLaunchKernelGGL(chnorm_apply, dim3(grid_for((int64_t)N * HW * C)), dim3(CN_THREADS), 0, st, x, gamma, beta,
                       mean, rstd, y, N, HW, C, groups, 0, act);
  }
  return check_launch("chnorm_fwd");
}

__global__ void gn_param_reduce(const float* __restrict__ part, int N, int C, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  for (int n = 0; n < N; ++n) {
    a += part[((int64_t)n * 2 + 0) * C + c];
    b += part[((int64_t)n * 2 + 1) * C + c];
  }
  dgamma[c] = a;
  dbeta[c] = b;
}

extern "C" int mdemi_chnorm_bwd(const float* dy, const float* x, const float* y, const float* mean, const float* rstd,
                                const float* gamma, const float* beta, float* dx, float* dgamma, float* dbeta,
                                int32_t N, int64_t HW, int32_t C, int32_t groups, int32_t is_bn, int32_t act,
                                void* workspace, void* stream) {
  (void)y;
  MDEMI_REQUIRE(dy && x && mean && rstd && gamma && beta && dx && dgamma && dbeta && N > 0 && HW > 0 && C > 0,
                "chnorm_bwd: bad args");
  if (!workspace) { set_error("chnorm_bwd: workspace required"); return MDEMI_EWORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)workspace;
  if (is_bn) {
    const int64_t rows = (int64_t)N * HW;
    const int rpb = rows_per_block(rows);
    const int nblk = (int)cdiv(rows, rpb);
    hipLaunchKernelGGL(bn_bwd_partial, dim3(nblk), dim3(CN_THREADS), 0, st, dy, x, mean, rstd, gamma, beta, part, rows,
                       C, act, rpb);
    hipLaunchKernelGGL(bn_bwd_combine, dim3((C + 255) / 256), dim3(256), 0, st, part, nblk, C, dgamma, dbeta);
    hipLaunchKernelGGL(bn_bwd_apply, dim3(grid_for(rows * C)), dim3(CN_THREADS), 0, st, dy, x, mean, rstd, gamma, beta,
                       dgamma, dbeta, dx, rows, C, act);
  } else {
    MDEMI_REQUIRE(groups > 0 && C % groups == 0, "chnorm_bwd: C %% groups != 0");
    hipLaunchKernelGGL(gn_bwd_kernel, dim3(N * groups), dim3(CN_THREADS), 0, st, dy, x, mean, rstd, gamma, beta, dx,
                       part, HW, C, groups, act);
    hipLaunchKernelGGL(gn_param_reduce, dim3((C + 255) / 256), dim3(256), 0, st, part, N, C, dgamma, dbeta);
  }
  return check_launch("chnorm_bwd");
}

// Inference-mode normalisation with given statistics (BatchNorm eval path:
// running stats folded into mean/rstd by the caller).
extern "C" int mdemi_chnorm_apply(const float* x, const float* gamma, const float* beta, const float* mean,
                                  const float* rstd, float* y, int32_t N, int64_t HW, int32_t C, int32_t groups,
                                  int32_t is_bn, int32_t act, void* stream) {
  MDEMI_REQUIRE(x && gamma && beta && mean && rstd && y && N > 0 && HW > 0 && C > 0, "chnorm_apply: bad args");
  const int G = is_bn ? C : groups;
  MDEMI_REQUIRE(G > 0 && C % G == 0, "chnorm_apply: bad groups");
  hipLaunchKernelGGL(chnorm_apply, dim3(grid_for((int64_t)N * HW * C)), dim3(CN_THREADS), 0, (hipStream_t)stream, x,
                     gamma, beta, mean, rstd, y, N, HW, C, G, is_bn, act);
  return check_launch("chnorm_apply");
}
