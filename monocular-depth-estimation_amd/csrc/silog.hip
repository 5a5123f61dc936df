// Scale-invariant log loss, restated (the reference's loss module is absent
// from the snapshot; its keys are loss.alpha / loss.beta / loss.per_image, e.g.
// json/nyu/newcrfs/newcrfs_github_eval.json, json/kitti/depthformer/
// depthformer_v8_cham_loss_per_image_4gpu.json).
//   g = log(pred) - log(gt) over gt > min_depth
//   L = alpha * sqrt(Var(g) + beta * mean(g)^2)   per image or per batch
// With biased Var and beta = 0.15 this is exactly NeW-CRFs' silog_loss
// sqrt(E[g^2] - 0.85 E[g]^2) * 10; unbiased=1 gives AdaBins' torch.var form.
// HBM-bound masked two-moment reduction; partial sums are combined in fp64.
#include "common.h"

namespace mdemi {

constexpr int SL_THREADS = 256;
constexpr int SL_MAXBLK = 128;  // per-image blocks

__global__ __launch_bounds__(SL_THREADS) void silog_partial(const float* __restrict__ pred,
                                                            const float* __restrict__ gt, float* __restrict__ part,
                                                            int64_t HW, float min_depth) {
  __shared__ float red[SL_THREADS / 64];
  const int b = blockIdx.y;
  const float* P = pred + (int64_t)b * HW;
  const float* G = gt + (int64_t)b * HW;
  float n = 0.f, s1 = 0.f, s2 = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * SL_THREADS + threadIdx.x; i < HW; i += (int64_t)gridDim.x * SL_THREADS) {
    const float gv = G[i];
    if (gv > min_depth) {
      const float d = logf(P[i]) - logf(gv);
      n += 1.f; s1 += d; s2 = fmaf(d, d, s2);
    }
  }
  n = block_sum<SL_THREADS>(n, red);
  s1 = block_sum<SL_THREADS>(s1, red);
  s2 = block_sum<SL_THREADS>(s2, red);
  if (threadIdx.x == 0) {
    float* o = part + ((int64_t)b * gridDim.x + blockIdx.x) * 3;
    o[0] = n; o[1] = s1; o[2] = s2;
  }
}

// stats[g] = {n, mean, D, sqrt(D)}; loss = mean_g alpha*sqrt(D_g).  One block: the
// partials of a group are summed by all threads in a fixed strided order, then a
// fixed fp64 tree through LDS (deterministic, no serial pass over B x nblk partials).
constexpr int SLF_THREADS = 256;
__global__ __launch_bounds__(SLF_THREADS) void silog_finalize(const float* __restrict__ part, int nblk, int B,
                                                              int per_image, int unbiased, float alpha, float beta,
                                                              float* __restrict__ loss, float* __restrict__ stats) {
  __shared__ double red[3][SLF_THREADS];
  const int t = threadIdx.x;
  const int G = per_image ? B : 1;
  double total = 0.0;
  int used = 0;
  for (int g = 0; g < G; ++g) {
    const int b0 = per_image ? g : 0, b1 = per_image ? g + 1 : B;
    const int64_t j0 = (int64_t)b0 * nblk, j1 = (int64_t)b1 * nblk;
    double n = 0, s1 = 0, s2 = 0;
    for (int64_t j = j0 + t; j < j1; j += SLF_THREADS) {
      const float* o = part + j * 3;
      n += o[0]; s1 += o[1]; s2 += o[2];
    }
    red[0][t] = n; red[1][t] = s1; red[2][t] = s2;
    __syncthreads();
    for (int w = SLF_THREADS / 2; w > 0; w >>= 1) {
      if (t < w) {
        red[0][t] += red[0][t + w]; red[1][t] += red[1][t + w]; red[2][t] += red[2][t + w];
      }
      __syncthreads();
    }
    if (t == 0) {
      n = red[0][0]; s1 = red[1][0]; s2 = red[2][0];
      double mean = n > 0 ? s1 / n : 0.0, D = 0.0;
      if (n > 0) {
        const double var = unbiased ? (n > 1 ? (s2 - n * mean * mean) / (n - 1) : 0.0) : (s2 / n - mean * mean);
        D = var + (double)beta * mean * mean;
        total += (double)alpha * sqrt(D > 0 ? D : 0.0);
        ++used;
      }
      stats[4 * g + 0] = (float)n;
      stats[4 * g + 1] = (float)mean;
      stats[4 * g + 2] = (float)D;
      stats[4 * g + 3] = (float)sqrt(D > 0 ? D : 0.0);
    }
    __syncthreads();
  }
  if (t == 0) loss[0] = used ? (float)(total / G) : 0.f;
}

__global__ __launch_bounds__(SL_THREADS) void silog_bwd_kernel(const float* __restrict__ pred,
                                                               const float* __restrict__ gt,
                                                               const float* __restrict__ stats,
                                                               const float* __restrict__ dloss,
                                                               float* __restrict__ dpred, int B, int64_t HW,
                                                               float min_depth, float alpha, float beta,
                                                               int per_image, int unbiased) {
  const int b = blockIdx.y;
  const int gidx = per_image ? b : 0;
  const int G = per_image ? B : 1;
  const float n = stats[4 * gidx + 0], mean = stats[4 * gidx + 1], sq = stats[4 * gidx + 3];
  // dL/dg_i = dloss/G * alpha / (2 sqrt(D)) * dD/dg_i
  const float coef = (n > 0.f && sq > 0.f) ? dloss[0] / (float)G * alpha / (2.f * sq) : 0.f;
  const float* P = pred + (int64_t)b * HW;
  const float* Gt = gt + (int64_t)b * HW;
  float* dP = dpred + (int64_t)b * HW;
  for (int64_t i = (int64_t)blockIdx.x * SL_THREADS + threadIdx.x; i < HW; i += (int64_t)gridDim.x * SL_THREADS) {
    const float gv = Gt[i];
    float out = 0.f;
    if (gv > min_depth) {
      const float pv = P[i];
      const float d = logf(pv) - logf(gv);
      float dD;
      if (unbiased) dD = 2.f * (d - mean) / (n - 1.f) + beta * 2.f * mean / n;
      else dD = 2.f * d / n - 2.f * (1.f - beta) * mean / n;
      out = coef * dD / pv;
    }
    dP[i] = out;
  }
}

static int sl_blocks(int64_t HW) {
  const int64_t nb = cdiv(HW, SL_THREADS * 4);
  return (int)(nb < SL_MAXBLK ? (nb < 1 ? 1 : nb) : SL_MAXBLK);
}

}  // namespace mdemi

using namespace mdemi;

extern "C" size_t mdemi_silog_workspace_size(int32_t B, int64_t HW) {
  return (size_t)B * sl_blocks(HW) * 3 * sizeof(float);
}

extern "C" int mdemi_silog_fwd(const float* pred, const float* gt, float* loss, float* stats, int32_t B, int64_t HW,
                               float min_depth, float alpha, float beta, int32_t per_image, int32_t unbiased,
                               void* workspace, void* stream) {
  MDEMI_REQUIRE(pred && gt && loss && stats && B > 0 && HW > 0, "silog_fwd: bad args");
  if (!workspace) { set_error("silog_fwd: workspace required"); return MDEMI_EWORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  const int nb = sl_blocks(HW);
  hipLaunchKernelGGL(silog_partial, dim3(nb, B), dim3(SL_THREADS), 0, st, pred, gt, (float*)workspace, HW, min_depth);
  hipLaunchKernelGGL(silog_finalize, dim3(1), dim3(SLF_THREADS), 0, st, (const float*)workspace, nb, B, per_image, unbiased,
                     alpha, beta, loss, stats);
  return check_launch("silog_fwd");
}

extern "C" int mdemi_silog_bwd(const float* pred, const float* gt, const float* stats, const float* dloss,
                               float* dpred, int32_t B, int64_t HW, float min_depth, float alpha, float beta,
                               int32_t per_image, int32_t unbiased, void* stream) {
  MDEMI_REQUIRE(pred && gt && stats && dloss && dpred && B > 0 && HW > 0, "silog_bwd: bad args");
  hipLaunchKernelGGL(silog_bwd_kernel, dim3(sl_blocks(HW), B), dim3(SL_THREADS), 0, (hipStream_t)stream, pred, gt,
                     stats, dloss, dpred, B, HW, min_depth, alpha, beta, per_image, unbiased);
  return check_launch("silog_bwd");
}
