// Kernels of the ODA2 ordered-swin2 family that the other model
// families do not already provide:
//
//   window_shuffle      roll + window_partition / window_reverse + roll back (+ residual)
//                       of PreNormOrderedSwinSA (oda2_red_order_swin2_decoder.py:83-85,
//                       103, 126-131) as one index-map sweep each way
//   ordered_softmax     softmax(scale * S + E[idx_i - idx_j + n - 1, head]) over each
//                       window's score rows (:87-92, 116-119) and its backward, with the
//                       depth-embedding gradient reduced per head
//   glu                 nn.GLU(dim=-1) of PreNormDWConvFF (oda2_red_order_reg_decoder.py:61,78)
//   pad_replicate       clamp-gather of an NHWC map (replicate padding and/or cropping:
//                       oda2_swin_transformer.py:12,258,287,327,491; the 5x5 depthwise
//                       conv's padding_mode="replicate", oda2_red_order_reg_decoder.py:65)
//                       and its adjoint (the fold of the padded gradient onto the edge)
//
// All of them are HBM sweeps: index maps and row-wise reductions, float4 over channels
// where the channel count allows.
#include "../../include/mdemi_ext.h"
#include "common.h"

namespace mdemi {

static unsigned grid_for(int64_t total, int per_block = 256) {
  int64_t b = cdiv(total, per_block);
  return (unsigned)(b < 65535 * 8 ? (b < 1 ? 1 : b) : 65535 * 8);
}

// window-major row r -> natural row of the rolled map:
//   r = ((n * nWh + wy) * nWw + wx) * ws^2 + ty * ws + tx,  natural (y, x) = ((wy*ws + ty + s) % H, ...)
__device__ __forceinline__ int64_t win_nat_row(int64_t r, int H, int W, int ws, int shift) {
  const int T = ws * ws;
  const int nWw = W / ws, nWh = H / ws;
  const int t = (int)(r % T);
  int64_t wi = r / T;
  const int wx = (int)(wi % nWw);
  wi /= nWw;
  const int wy = (int)(wi % nWh);
  const int64_t n = wi / nWh;
  int y = wy * ws + t / ws + shift, x = wx * ws + t % ws + shift;
  if (y >= H) y -= H;
  if (x >= W) x -= W;
  return (n * H + y) * W + x;
}

template <typename V>
__global__ __launch_bounds__(256) void win_shuffle_kernel(const V* __restrict__ src, V* __restrict__ dst,
                                                          const V* __restrict__ add, int64_t rows, int cv, int H,
                                                          int W, int ws, int shift, int inverse) {
  const int64_t total = rows * cv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / cv;
    const int c = (int)(e % cv);
    const int64_t nat = win_nat_row(r, H, W, ws, shift);
    if (!inverse) {
      dst[r * cv + c] = src[nat * cv + c];
    } else {
      V v = src[r * cv + c];
      if (add) v = v + add[nat * cv + c];
      dst[nat * cv + c] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// ordered softmax.  Layout: S / P / dP / dS are [nwin][heads][T][T] (T = ws^2 tokens,
// 64 or 256), idx is [nwin][T] (window-major depth indices), table is the reference's
// depth_embedding [2n-1][heads].  One workgroup = one head x a strided set of windows;
// each wave owns score rows, lane j holds columns j, j+64, ...
// ---------------------------------------------------------------------------
constexpr int OS_MAXTAB = 511;  // 2 * num_emb - 1 with num_emb <= 256

template <int T>
// S and P (forward) and dP and dS (backward) may alias: each row is read whole before it is
// written, so neither pair is __restrict__.  Depth indices are clamped to [0, nemb-1] as they
// are staged: the reference's floor(sigmoid(logit) * n - 1e-3) gives -1 where the sigmoid
// underflows to 0 (logit < -88), and F.embedding raises there; the clamp keeps every table
// and histogram access inside its LDS array instead of reading or adding out of bounds.
__global__ __launch_bounds__(256) void ordered_softmax_fwd_kernel(const float* S, float* P,
                                                                  const int* __restrict__ idx,
                                                                  const float* __restrict__ table, int nwin,
                                                                  int heads, int nemb, float scale) {
  constexpr int Q = T / 64;
  __shared__ float tab[OS_MAXTAB + 1];
  __shared__ int widx[T];
  const int h = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ntab = 2 * nemb - 1;
  for (int k = threadIdx.x; k < ntab; k += 256) tab[k] = table ? table[(int64_t)k * heads + h] : 0.f;
  for (int w = blockIdx.y; w < nwin; w += gridDim.y) {
    __syncthreads();
    for (int t = threadIdx.x; t < T; t += 256) widx[t] = table ? min(max(idx[(int64_t)w * T + t], 0), nemb - 1) : 0;
    __syncthreads();
    const int64_t base = ((int64_t)w * heads + h) * T * T;
    for (int row = wv; row < T; row += 4) {
      const float* s = S + base + (int64_t)row * T;
      const int off = widx[row] + nemb - 1;
      float v[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int j = lane + 64 * q;
        v[q] = fmaf(s[j], scale, tab[off - widx[j]]);
      }
      float m = v[0];
#pragma unroll
      for (int q = 1; q < Q; ++q) m = fmaxf(m, v[q]);
      m = wave_max(m);
      float l = 0.f;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        v[q] = __expf(v[q] - m);
        l += v[q];
      }
      const float inv = 1.f / wave_sum(l);
      float* p = P + base + (int64_t)row * T;
#pragma unroll
      for (int q = 0; q < Q; ++q) p[lane + 64 * q] = v[q] * inv;
    }
  }
}

// dZ = P o (dP - rowsum(P o dP)); dS = scale * dZ; per-block histogram of dZ by
// relative index into part[blockIdx.y][k * heads + h] (the table's own layout)
template <int T>
__global__ __launch_bounds__(256) void ordered_softmax_bwd_kernel(const float* __restrict__ P,
                                                                  const float* dP, float* dS,
                                                                  const int* __restrict__ idx, float* __restrict__ part,
                                                                  int nwin, int heads, int nemb, float scale) {
  constexpr int Q = T / 64;
  __shared__ float hist[OS_MAXTAB + 1];
  __shared__ int widx[T];
  const int h = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ntab = 2 * nemb - 1;
  const bool tab = part != nullptr;
  for (int k = threadIdx.x; k < ntab; k += 256) hist[k] = 0.f;
  for (int w = blockIdx.y; w < nwin; w += gridDim.y) {
    __syncthreads();
    if (tab)
      for (int t = threadIdx.x; t < T; t += 256) widx[t] = min(max(idx[(int64_t)w * T + t], 0), nemb - 1);
    __syncthreads();
    const int64_t base = ((int64_t)w * heads + h) * T * T;
    for (int row = wv; row < T; row += 4) {
      const int64_t o = base + (int64_t)row * T;
      float p[Q], g[Q];
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        p[q] = P[o + lane + 64 * q];
        g[q] = dP[o + lane + 64 * q];
        d = fmaf(p[q], g[q], d);
      }
      d = wave_sum(d);
      const int off = tab ? widx[row] + nemb - 1 : 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const float dz = p[q] * (g[q] - d);
        dS[o + lane + 64 * q] = dz * scale;
        if (tab) atomicAdd(&hist[off - widx[lane + 64 * q]], dz);
      }
    }
  }
  if (!tab) return;
  __syncthreads();
  for (int k = threadIdx.x; k < ntab; k += 256) part[(int64_t)blockIdx.y * ntab * heads + (int64_t)k * heads + h] = hist[k];
}

static int os_blocks_y(int nwin, int heads) {
  int by = (2048 + heads - 1) / heads;
  return nwin < by ? nwin : by;
}

// ---------------------------------------------------------------------------
// GLU: y[m][f] = x[m][f] * sigmoid(x[m][F + f])
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void glu_fwd_kernel(const float4* __restrict__ x, float4* __restrict__ y, int64_t M,
                                                      int F4) {
  const int64_t total = M * F4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / F4;
    const int f = (int)(e % F4);
    const float4 a = x[m * 2 * F4 + f], b = x[m * 2 * F4 + F4 + f];
    y[e] = make_float4(a.x * sigmoid_f(b.x), a.y * sigmoid_f(b.y), a.z * sigmoid_f(b.z), a.w * sigmoid_f(b.w));
  }
}

__global__ __launch_bounds__(256) void glu_bwd_kernel(const float4* __restrict__ x, const float4* __restrict__ dy,
                                                      float4* __restrict__ dx, int64_t M, int F4) {
  const int64_t total = M * F4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / F4;
    const int f = (int)(e % F4);
    const float4 a = x[m * 2 * F4 + f], b = x[m * 2 * F4 + F4 + f], g = dy[e];
    float4 da, db;
    float s;
    s = sigmoid_f(b.x); da.x = g.x * s; db.x = g.x * a.x * s * (1.f - s);
    s = sigmoid_f(b.y); da.y = g.y * s; db.y = g.y * a.y * s * (1.f - s);
    s = sigmoid_f(b.z); da.z = g.z * s; db.z = g.z * a.z * s * (1.f - s);
    s = sigmoid_f(b.w); da.w = g.w * s; db.w = g.w * a.w * s * (1.f - s);
    dx[m * 2 * F4 + f] = da;
    dx[m * 2 * F4 + F4 + f] = db;
  }
}

// ---------------------------------------------------------------------------
// clamp-gather: y[n][oy][ox] = x[n][clamp(oy - pt, 0, H-1)][clamp(ox - pl, 0, W-1)]
// adjoint:     dx[n][y][x]  = sum of dy over the (oy, ox) that clamp to (y, x)
// ---------------------------------------------------------------------------
template <typename V>
__global__ __launch_bounds__(256) void pad_rep_kernel(const V* __restrict__ x, V* __restrict__ y, int N, int H, int W,
                                                      int cv, int OH, int OW, int pt, int pl) {
  const int64_t total = (int64_t)N * OH * OW * cv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c = (int)(e % cv);
    int64_t r = e / cv;
    const int ox = (int)(r % OW);
    r /= OW;
    const int oy = (int)(r % OH);
    const int64_t n = r / OH;
    const int iy = min(max(oy - pt, 0), H - 1), ix = min(max(ox - pl, 0), W - 1);
    y[e] = x[((n * H + iy) * W + ix) * cv + c];
  }
}

__device__ __forceinline__ void fold_range(int i, int n_in, int n_out, int p, int& lo, int& hi) {
  lo = i == 0 ? 0 : i + p;
  hi = i == n_in - 1 ? n_out - 1 : i + p;
  lo = max(lo, 0);
  hi = min(hi, n_out - 1);
}

template <typename V>
__global__ __launch_bounds__(256) void pad_fold_rep_kernel(const V* __restrict__ dy, V* __restrict__ dx, int N, int H,
                                                           int W, int cv, int OH, int OW, int pt, int pl) {
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c = (int)(e % cv);
    int64_t r = e / cv;
    const int x = (int)(r % W);
    r /= W;
    const int yy = (int)(r % H);
    const int64_t n = r / H;
    int y0, y1, x0, x1;
    fold_range(yy, H, OH, pt, y0, y1);
    fold_range(x, W, OW, pl, x0, x1);
    V acc = V{};
    for (int oy = y0; oy <= y1; ++oy)
      for (int ox = x0; ox <= x1; ++ox) acc = acc + dy[((n * OH + oy) * OW + ox) * cv + c];
    dx[e] = acc;
  }
}

}  // namespace mdemi

using namespace mdemi;

extern "C" int mdemi_window_shuffle(const float* src, float* dst, const float* add, int32_t N, int32_t H, int32_t W,
                                    int32_t C, int32_t ws, int32_t shift, int32_t inverse, void* stream) {
  MDEMI_REQUIRE(src && dst && N > 0 && C > 0 && ws > 0 && H > 0 && W > 0, "window_shuffle: bad args");
  MDEMI_REQUIRE(H % ws == 0 && W % ws == 0, "window_shuffle: %dx%d is not a multiple of the window %d", H, W, ws);
  MDEMI_REQUIRE(shift >= 0 && shift < ws, "window_shuffle: bad shift %d", shift);
  MDEMI_REQUIRE(!add || inverse, "window_shuffle: the residual add is for the inverse (scatter) direction");
  const int64_t rows = (int64_t)N * H * W;
  hipStream_t st = (hipStream_t)stream;
  const bool v4 = C % 4 == 0 && (((uintptr_t)src | (uintptr_t)dst | (uintptr_t)add) & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(win_shuffle_kernel<float4>, dim3(grid_for(rows * (C / 4))), dim3(256), 0, st,
                       (const float4*)src, (float4*)dst, (const float4*)add, rows, C / 4, H, W, ws, shift, inverse);
  else
    hipLaunchKernelGGL(win_shuffle_kernel<float>, dim3(grid_for(rows * C)), dim3(256), 0, st, src, dst, add, rows, C,
                       H, W, ws, shift, inverse);
  return check_launch("window_shuffle");
}

extern "C" int mdemi_window_shuffle_i32(const int32_t* src, int32_t* dst, int32_t N, int32_t H, int32_t W,
                                        int32_t ws, int32_t shift, void* stream) {
  MDEMI_REQUIRE(src && dst && N > 0 && ws > 0 && H > 0 && W > 0 && H % ws == 0 && W % ws == 0 && shift >= 0 &&
                    shift < ws,
                "window_shuffle_i32: bad args");
  const int64_t rows = (int64_t)N * H * W;
  hipLaunchKernelGGL(win_shuffle_kernel<int>, dim3(grid_for(rows)), dim3(256), 0, (hipStream_t)stream, src, dst,
                     (const int*)nullptr, rows, 1, H, W, ws, shift, 0);
  return check_launch("window_shuffle_i32");
}

#define OS_DISPATCH(KERNEL, ...)                                                                  \
  do {                                                                                            \
    if (T == 64) hipLaunchKernelGGL(KERNEL<64>, grid, dim3(256), 0, st, __VA_ARGS__);             \
    else hipLaunchKernelGGL(KERNEL<256>, grid, dim3(256), 0, st, __VA_ARGS__);                    \
  } while (0)

extern "C" int mdemi_ordered_softmax_fwd(const float* S, float* P, const int32_t* idx, const float* table, int32_t nwin,
                                         int32_t heads, int32_t T, int32_t num_emb, float scale, void* stream) {
  MDEMI_REQUIRE(S && P && nwin > 0 && heads > 0, "ordered_softmax_fwd: bad args");
  MDEMI_REQUIRE(T == 64 || T == 256, "ordered_softmax_fwd: windows of 8x8 or 16x16 tokens only (T=%d)", T);
  MDEMI_REQUIRE(!table || (idx && num_emb > 0 && 2 * num_emb - 1 <= OS_MAXTAB),
                "ordered_softmax_fwd: bias needs indices and 1 <= num_emb <= 256");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)heads, (unsigned)os_blocks_y(nwin, heads));
  OS_DISPATCH(ordered_softmax_fwd_kernel, S, P, (const int*)idx, table, nwin, heads, table ? num_emb : 1, scale);
  return check_launch("ordered_softmax_fwd");
}

extern "C" size_t mdemi_ordered_softmax_bwd_workspace_size(int32_t nwin, int32_t heads, int32_t num_emb) {
  const int64_t by = os_blocks_y(nwin, heads), cols = (int64_t)(2 * num_emb - 1) * heads;
  return align_up((size_t)(by * cols) * sizeof(float), 256) + colsum_ws_bytes(by, cols);
}

extern "C" int mdemi_ordered_softmax_bwd(const float* P, const float* dP, float* dS, const int32_t* idx,
                                         float* d_table, int32_t nwin, int32_t heads, int32_t T, int32_t num_emb,
                                         float scale, void* workspace, void* stream) {
  MDEMI_REQUIRE(P && dP && dS && nwin > 0 && heads > 0, "ordered_softmax_bwd: bad args");
  MDEMI_REQUIRE(T == 64 || T == 256, "ordered_softmax_bwd: windows of 8x8 or 16x16 tokens only (T=%d)", T);
  MDEMI_REQUIRE(!d_table || (idx && num_emb > 0 && 2 * num_emb - 1 <= OS_MAXTAB),
                "ordered_softmax_bwd: bias gradient needs indices and 1 <= num_emb <= 256");
  if (d_table && !workspace) { set_error("ordered_softmax_bwd: workspace required"); return MDEMI_EWORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  const int by = os_blocks_y(nwin, heads);
  dim3 grid((unsigned)heads, (unsigned)by);
  float* part = d_table ? (float*)workspace : nullptr;
  OS_DISPATCH(ordered_softmax_bwd_kernel, P, dP, dS, (const int*)idx, part, nwin, heads, d_table ? num_emb : 1, scale);
  if (d_table) {
    const int64_t cols = (int64_t)(2 * num_emb - 1) * heads;
    void* cws = (char*)workspace + align_up((size_t)(by * cols) * sizeof(float), 256);
    int rc = colsum_launch(part, by, cols, cols, d_table, 0, cws, st);
    if (rc) return rc;
  }
  return check_launch("ordered_softmax_bwd");
}

extern "C" int mdemi_glu_fwd(const float* x, float* y, int64_t M, int32_t F, void* stream) {
  MDEMI_REQUIRE(x && y && M > 0 && F > 0 && F % 4 == 0, "glu_fwd: bad args (F %% 4 == 0)");
  hipLaunchKernelGGL(glu_fwd_kernel, dim3(grid_for(M * (F / 4))), dim3(256), 0, (hipStream_t)stream,
                     (const float4*)x, (float4*)y, M, F / 4);
  return check_launch("glu_fwd");
}

extern "C" int mdemi_glu_bwd(const float* x, const float* dy, float* dx, int64_t M, int32_t F, void* stream) {
  MDEMI_REQUIRE(x && dy && dx && M > 0 && F > 0 && F % 4 == 0, "glu_bwd: bad args (F %% 4 == 0)");
  hipLaunchKernelGGL(glu_bwd_kernel, dim3(grid_for(M * (F / 4))), dim3(256), 0, (hipStream_t)stream,
                     (const float4*)x, (const float4*)dy, (float4*)dx, M, F / 4);
  return check_launch("glu_bwd");
}

extern "C" int mdemi_pad_replicate(const float* x, float* y, int32_t N, int32_t H, int32_t W, int32_t C, int32_t OH,
                                   int32_t OW, int32_t pt, int32_t pl, int32_t inverse, void* stream) {
  MDEMI_REQUIRE(x && y && N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0 && pt >= 0 && pl >= 0,
                "pad_replicate: bad args");
  hipStream_t st = (hipStream_t)stream;
  const bool v4 = C % 4 == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0;
  const int cv = v4 ? C / 4 : C;
  const int64_t total = (int64_t)N * (inverse ? (int64_t)H * W : (int64_t)OH * OW) * cv;
  if (!inverse) {
    if (v4)
      hipLaunchKernelGGL(pad_rep_kernel<float4>, dim3(grid_for(total)), dim3(256), 0, st, (const float4*)x,
                         (float4*)y, N, H, W, cv, OH, OW, pt, pl);
    else
      hipLaunchKernelGGL(pad_rep_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, x, y, N, H, W, cv, OH, OW,
                         pt, pl);
  } else {  // x = dy [N][OH][OW][C] -> y = dx [N][H][W][C]
    if (v4)
      hipLaunchKernelGGL(pad_fold_rep_kernel<float4>, dim3(grid_for(total)), dim3(256), 0, st, (const float4*)x,
                         (float4*)y, N, H, W, cv, OH, OW, pt, pl);
    else
      hipLaunchKernelGGL(pad_fold_rep_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, x, y, N, H, W, cv, OH,
                         OW, pt, pl);
  }
  return check_launch("pad_replicate");
}
