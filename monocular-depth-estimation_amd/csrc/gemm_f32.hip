// fp32 GEMM on gfx950 MFMA (v_mfma_f32_32x32x2_f32: exact f32 products,
// f32 accumulate, 64 FLOP/clk/SIMD = the chip's 157 TF fp32 matrix peak).
//
// One kernel family serves every dense contraction of the hot path:
//   nn.Linear fwd / dgrad / wgrad   (swin_transformer.py:18-20,104,106,259;
//                                     newcrf_layers.py:16-20,102,104; ...)
//   nn.Conv2d fwd / dgrad / wgrad   through an implicit-im2col operand
//                                     (newcrf_layers.py:384,389;
//                                      uper_crf_head.py:38-44,341-348; ...)
// Operand element (i,k) of A / (k,j) of B is produced by a loader selected at
// compile time (dense k-contiguous, dense m/n-contiguous, or NHWC conv gather)
// with an optional GELU transform on load (so nn.GELU's output is never
// materialised: fc2 reads GELU(fc1 pre-activation) directly).  The epilogue
// fuses alpha/beta, bias, activation (or GELU-backward multiply) and a
// residual add.  Long reductions (weight gradients over B*H*W rows) split K
// over workgroups into fp32 slabs reduced by a second deterministic kernel.
//
// Tiling: 128x128 block tile, BK = 16, 256 threads = 4 waves in 2x2, each wave
// 64x64 = 2x2 MFMA 32x32 accumulators (64 AGPRs).  Register-staged double-
// buffered LDS ([k][m] / [k][n] images, 32 consecutive floats per half-wave
// fragment read: conflict-free), one barrier per K tile.
#include "common.h"

namespace mdemi {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int GBM = 128, GBN = 128, GBK = 16, GTHREADS = 256;

struct GemmParams {
  int M, N, K, batch, split, ktile_per_split;
  const float* A; int64_t lda, a_bs;
  const float* B; int64_t ldb, b_bs;
  float* C; int64_t ldc, c_bs;
  float alpha, beta;
  const float* bias; int bias_mode, act;
  const float* aux; int64_t ldaux, aux_bs;
  const float* res; int64_t ldres, res_bs;
  float* slab;  // split-K partials [split][batch][M][N]
  mdemi_conv_geom cv;
  int a_vec, b_vec;  // 1: 16-byte vector loads legal for this operand
};

// LDS row pitch per operand layout: MN-contiguous images are written with
// ds_write_b128 (pitch must stay 16-B aligned); K-contiguous sources are
// transposed with 4x ds_write_b32 (pitch 130 spreads the 4 k-rows a 32-lane
// group writes over distinct banks).
template <int LAYOUT>
struct Pitch { static constexpr int v = (LAYOUT == MDEMI_L_MNCONTIG) ? GBM + 4 : GBM + 2; };

__device__ __forceinline__ float4 ld4_guard(const float* p, int n_valid, bool vec) {
  // n_valid: number of leading elements inside the tensor (0..4)
  if (n_valid >= 4 && vec) return *reinterpret_cast<const float4*>(p);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n_valid > 0) r.x = p[0];
  if (n_valid > 1) r.y = p[1];
  if (n_valid > 2) r.z = p[2];
  if (n_valid > 3) r.w = p[3];
  return r;
}

template <int OP>
__device__ __forceinline__ float4 apply_op(float4 v) {
  if (OP == MDEMI_OP_GELU) { v.x = gelu_f(v.x); v.y = gelu_f(v.y); v.z = gelu_f(v.z); v.w = gelu_f(v.w); }
  return v;
}

// ---------------------------------------------------------------------------
// Operand loaders.  Each thread stages 2 float4 per operand per K tile.
//   K-contiguous tile  (128 rows x 16 k): f = t + 256 r -> row f>>2, k-quad f&3
//   MN-contiguous tile (16 k x 128 cols): f = t + 256 r -> k f>>5, col-quad f&31
// `rows`/`ld`: for A rows are i (M), for B rows are j (N).
// ---------------------------------------------------------------------------
template <int LAYOUT, int OP>
struct Loader;

// dense [row][k]
template <int OP>
struct Loader<MDEMI_L_KCONTIG, OP> {
  const float* base; int64_t ld; int rows, K; bool vec;
  int row[2]; int kq;
  __device__ void init(const float* p, int64_t ld_, int rows_, int K_, bool vec_, int row0, int t,
                       const mdemi_conv_geom&) {
    base = p; ld = ld_; rows = rows_; K = K_; vec = vec_;
    row[0] = row0 + (t >> 2); row[1] = row0 + 64 + (t >> 2); kq = t & 3;
  }
  __device__ void load(int k0, float4 (&r)[2]) const {
    const int k = k0 + 4 * kq;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int nv = (row[s] < rows) ? min(4, K - k) : 0;
      r[s] = apply_op<OP>(ld4_guard(base + (int64_t)row[s] * ld + k, nv, vec));
    }
  }
  __device__ static void store(float* lds, int t, const float4 (&r)[2]) {
    constexpr int P = Pitch<MDEMI_L_KCONTIG>::v;
    const int kq = t & 3;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int rl = (t >> 2) + 64 * s;
      lds[(4 * kq + 0) * P + rl] = r[s].x;
      lds[(4 * kq + 1) * P + rl] = r[s].y;
      lds[(4 * kq + 2) * P + rl] = r[s].z;
      lds[(4 * kq + 3) * P + rl] = r[s].w;
    }
  }
};

// dense [k][row]
template <int OP>
struct Loader<MDEMI_L_MNCONTIG, OP> {
  const float* base; int64_t ld; int rows, K; bool vec;
  int col; int kl;
  __device__ void init(const float* p, int64_t ld_, int rows_, int K_, bool vec_, int row0, int t,
                       const mdemi_conv_geom&) {
    base = p; ld = ld_; rows = rows_; K = K_; vec = vec_;
    col = row0 + 4 * (t & 31); kl = t >> 5;
  }
  __device__ void load(int k0, float4 (&r)[2]) const {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k = k0 + kl + 8 * s;
      const int nv = (k < K) ? min(4, rows - col) : 0;
      r[s] = apply_op<OP>(ld4_guard(base + (int64_t)k * ld + col, nv, vec));
    }
  }
  __device__ static void store(float* lds, int t, const float4 (&r)[2]) {
    constexpr int P = Pitch<MDEMI_L_MNCONTIG>::v;
#pragma unroll
    for (int s = 0; s < 2; ++s)
      *reinterpret_cast<float4*>(lds + ((t >> 5) + 8 * s) * P + 4 * (t & 31)) = r[s];
  }
};

// Implicit im2col of an NHWC activation, operand A (k-contiguous role):
// A(i, k) = X[n, oy*s - p + ky, ox*s - p + kx, c], i = (n,oy,ox), k = (ky,kx,c).
// Requires C % 4 == 0 so a k-quad never straddles a filter tap.
template <int OP>
struct ConvLoaderA {
  const float* base; mdemi_conv_geom g; int rows, K; int kq;
  int n[2], iy0[2], ix0[2]; bool valid[2];
  __device__ void init(const float* p, int64_t, int rows_, int K_, bool, int row0, int t,
                       const mdemi_conv_geom& g_) {
    base = p; g = g_; rows = rows_; K = K_; kq = t & 3;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = row0 + (t >> 2) + 64 * s;
      valid[s] = i < rows;
      const int ii = valid[s] ? i : 0;
      const int ox = ii % g.ow, tmp = ii / g.ow;
      const int oy = tmp % g.oh;
      n[s] = tmp / g.oh;
      iy0[s] = oy * g.stride - g.pad;
      ix0[s] = ox * g.stride - g.pad;
    }
  }
  __device__ void load(int k0, float4 (&r)[2]) const {
    const int k = k0 + 4 * kq;
    const bool kin = k < K;
    const int kk = kin ? k : 0;
    const int c = kk % g.c, tap = kk / g.c;
    const int kx = tap % g.kw, ky = tap / g.kw;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      int iy = iy0[s] + ky, ix = ix0[s] + kx;
      bool ok = kin && valid[s];
      if (g.pad_mode == MDEMI_PAD_REPLICATE) {
        iy = min(max(iy, 0), g.h - 1); ix = min(max(ix, 0), g.w - 1);
      } else {
        ok = ok && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
      }
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok) v = *reinterpret_cast<const float4*>(base + (((int64_t)n[s] * g.h + iy) * g.w + ix) * g.c + c);
      r[s] = apply_op<OP>(v);
    }
  }
  __device__ static void store(float* lds, int t, const float4 (&r)[2]) {
    Loader<MDEMI_L_KCONTIG, OP>::store(lds, t, r);
  }
};

// Implicit im2col, operand B (n-contiguous role, weight gradients):
// B(k, j) = X[n, oy*s - p + ky, ox*s - p + kx, c], k = (n,oy,ox), j = (ky,kx,c).
template <int OP>
struct ConvLoaderB {
  const float* base; mdemi_conv_geom g; int cols, K; int kl;
  int c, ky, kx; bool jvalid;
  __device__ void init(const float* p, int64_t, int cols_, int K_, bool, int col0, int t,
                       const mdemi_conv_geom& g_) {
    base = p; g = g_; cols = cols_; K = K_; kl = t >> 5;
    const int j = col0 + 4 * (t & 31);
    jvalid = j < cols;
    const int jj = jvalid ? j : 0;
    c = jj % g.c; const int tap = jj / g.c; kx = tap % g.kw; ky = tap / g.kw;
  }
  __device__ void load(int k0, float4 (&r)[2]) const {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k = k0 + kl + 8 * s;
      bool ok = jvalid && k < K;
      const int kk = ok ? k : 0;
      const int ox = kk % g.ow, tmp = kk / g.ow;
      const int oy = tmp % g.oh, nn = tmp / g.oh;
      int iy = oy * g.stride - g.pad + ky, ix = ox * g.stride - g.pad + kx;
      if (g.pad_mode == MDEMI_PAD_REPLICATE) {
        iy = min(max(iy, 0), g.h - 1); ix = min(max(ix, 0), g.w - 1);
      } else {
        ok = ok && iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
      }
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok) v = *reinterpret_cast<const float4*>(base + (((int64_t)nn * g.h + iy) * g.w + ix) * g.c + c);
      r[s] = apply_op<OP>(v);
    }
  }
  __device__ static void store(float* lds, int t, const float4 (&r)[2]) {
    Loader<MDEMI_L_MNCONTIG, OP>::store(lds, t, r);
  }
};

template <int LAYOUT, int OP, bool IS_A>
struct PickLoader { using T = Loader<LAYOUT, OP>; };
template <int OP>
struct PickLoader<MDEMI_L_CONV, OP, true> { using T = ConvLoaderA<OP>; };
template <int OP>
struct PickLoader<MDEMI_L_CONV, OP, false> { using T = ConvLoaderB<OP>; };

// LDS pitch of the staged image: the conv A loader writes like a K-contiguous
// operand, the conv B loader like an MN-contiguous one.
template <int LAYOUT, bool IS_A>
struct StagePitch {
  static constexpr int v = (LAYOUT == MDEMI_L_CONV) ? (IS_A ? Pitch<MDEMI_L_KCONTIG>::v : Pitch<MDEMI_L_MNCONTIG>::v)
                                                    : Pitch<LAYOUT>::v;
};

__device__ __forceinline__ float epilogue_value(const GemmParams& p, int b, int i, int j, float acc) {
  float v = p.alpha * acc;
  if (p.beta != 0.f) v += p.beta * p.C[(int64_t)b * p.c_bs + (int64_t)i * p.ldc + j];
  if (p.bias_mode == MDEMI_BIAS_COL) v += p.bias[j];
  else if (p.bias_mode == MDEMI_BIAS_ROW) v += p.bias[i];
  if (p.act == MDEMI_ACT_GELU_GRAD) v *= gelu_grad_f(p.aux[(int64_t)b * p.aux_bs + (int64_t)i * p.ldaux + j]);
  else if (p.act != MDEMI_ACT_NONE) v = apply_act(p.act, v);
  if (p.res) v += p.res[(int64_t)b * p.res_bs + (int64_t)i * p.ldres + j];
  return v;
}

template <int AL, int BL, int AOP, int BOP>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_f32_kernel(GemmParams p) {
  constexpr int PA = StagePitch<AL, true>::v;
  constexpr int PB = StagePitch<BL, false>::v;
  __shared__ __attribute__((aligned(16))) float As[2][GBK * PA];
  __shared__ __attribute__((aligned(16))) float Bs[2][GBK * PB];

  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int zb = blockIdx.z;
  const int b = zb / p.split, sidx = zb % p.split;
  const int bm = blockIdx.y * GBM, bn = blockIdx.x * GBN;

  typename PickLoader<AL, AOP, true>::T la;
  typename PickLoader<BL, BOP, false>::T lb;
  la.init(p.A + (int64_t)b * p.a_bs, p.lda, p.M, p.K, p.a_vec, bm, t, p.cv);
  lb.init(p.B + (int64_t)b * p.b_bs, p.ldb, p.N, p.K, p.b_vec, bn, t, p.cv);

  const int ktiles_total = (p.K + GBK - 1) / GBK;
  const int kt_begin = sidx * p.ktile_per_split;
  const int kt_end = min(ktiles_total, kt_begin + p.ktile_per_split);

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  float4 ra[2], rb[2];
  int cur = 0;
  if (kt_begin < kt_end) {
    la.load(kt_begin * GBK, ra);
    lb.load(kt_begin * GBK, rb);
    la.store(As[0], t, ra);
    lb.store(Bs[0], t, rb);
  }
  __syncthreads();

  const int l31 = lane & 31, h = lane >> 5;
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const bool more = kt + 1 < kt_end;
    if (more) {
      la.load((kt + 1) * GBK, ra);
      lb.load((kt + 1) * GBK, rb);
    }
    const float* a_s = As[cur];
    const float* b_s = Bs[cur];
#pragma unroll
    for (int kk = 0; kk < GBK / 2; ++kk) {
      const int krow = 2 * kk + h;
      const float a0 = a_s[krow * PA + wm * 64 + l31];
      const float a1 = a_s[krow * PA + wm * 64 + 32 + l31];
      const float b0 = b_s[krow * PB + wn * 64 + l31];
      const float b1 = b_s[krow * PB + wn * 64 + 32 + l31];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (more) {
      la.store(As[cur ^ 1], t, ra);
      lb.store(Bs[cur ^ 1], t, rb);
    }
    __syncthreads();
    cur ^= 1;
  }

  // Epilogue.  acc[tm][tn][r] holds C(row, col) with
  //   row = bm + wm*64 + tm*32 + (r&3) + 8*(r>>2) + 4*h,  col = bn + wn*64 + tn*32 + l31
  if (p.split > 1) {
    float* S = p.slab + ((int64_t)sidx * p.batch + b) * (int64_t)p.M * p.N;
#pragma unroll
    for (int tm = 0; tm < 2; ++tm)
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) {
        const int j = bn + wn * 64 + tn * 32 + l31;
        if (j >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = bm + wm * 64 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (i < p.M) S[(int64_t)i * p.N + j] = acc[tm][tn][r];
        }
      }
    return;
  }
  float* Cb = p.C + (int64_t)b * p.c_bs;
#pragma unroll
  for (int tm = 0; tm < 2; ++tm)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int j = bn + wn * 64 + tn * 32 + l31;
      if (j >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = bm + wm * 64 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (i < p.M) Cb[(int64_t)i * p.ldc + j] = epilogue_value(p, b, i, j, acc[tm][tn][r]);
      }
    }
}

// Deterministic split-K combine + epilogue: sums slabs in split order.
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemmParams p) {
  const int64_t MN = (int64_t)p.M * p.N;
  const int64_t total = MN * p.batch;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / MN);
    const int64_t rem = e - (int64_t)b * MN;
    const int i = (int)(rem / p.N), j = (int)(rem - (int64_t)i * p.N);
    float s = 0.f;
    for (int q = 0; q < p.split; ++q) s += p.slab[((int64_t)q * p.batch + b) * MN + rem];
    p.C[(int64_t)b * p.c_bs + (int64_t)i * p.ldc + j] = epilogue_value(p, b, i, j, s);
  }
}

using KernelFn = void (*)(GemmParams);

template <int AL, int BL>
static KernelFn pick_ops(int aop, int bop) {
  if (aop == MDEMI_OP_NONE && bop == MDEMI_OP_NONE) return gemm_f32_kernel<AL, BL, MDEMI_OP_NONE, MDEMI_OP_NONE>;
  if (aop == MDEMI_OP_GELU && bop == MDEMI_OP_NONE && AL == MDEMI_L_KCONTIG)
    return gemm_f32_kernel<AL, BL, MDEMI_OP_GELU, MDEMI_OP_NONE>;
  if (aop == MDEMI_OP_NONE && bop == MDEMI_OP_GELU && BL == MDEMI_L_MNCONTIG)
    return gemm_f32_kernel<AL, BL, MDEMI_OP_NONE, MDEMI_OP_GELU>;
  return nullptr;
}

static KernelFn pick_kernel(int al, int bl, int aop, int bop) {
#define MDEMI_PICK(X, Y) \
  if (al == X && bl == Y) return pick_ops<X, Y>(aop, bop);
  MDEMI_PICK(MDEMI_L_KCONTIG, MDEMI_L_KCONTIG)
  MDEMI_PICK(MDEMI_L_KCONTIG, MDEMI_L_MNCONTIG)
  MDEMI_PICK(MDEMI_L_MNCONTIG, MDEMI_L_KCONTIG)
  MDEMI_PICK(MDEMI_L_MNCONTIG, MDEMI_L_MNCONTIG)
  MDEMI_PICK(MDEMI_L_CONV, MDEMI_L_KCONTIG)
  MDEMI_PICK(MDEMI_L_CONV, MDEMI_L_MNCONTIG)
  MDEMI_PICK(MDEMI_L_MNCONTIG, MDEMI_L_CONV)
  MDEMI_PICK(MDEMI_L_KCONTIG, MDEMI_L_CONV)
#undef MDEMI_PICK
  return nullptr;
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static int validate(const mdemi_gemm_desc* d) {
  MDEMI_REQUIRE(d, "gemm: null descriptor");
  MDEMI_REQUIRE(d->M > 0 && d->N > 0 && d->K > 0 && d->batch > 0, "gemm: bad sizes M=%d N=%d K=%d batch=%d",
                d->M, d->N, d->K, d->batch);
  MDEMI_REQUIRE(d->A && d->B && d->C, "gemm: null operand");
  MDEMI_REQUIRE(d->split_k >= 1, "gemm: split_k must be >= 1");
  if (d->a_layout == MDEMI_L_CONV || d->b_layout == MDEMI_L_CONV) {
    const mdemi_conv_geom& g = d->conv;
    MDEMI_REQUIRE(g.c % 4 == 0, "gemm: conv operand needs C %% 4 == 0 (C=%d)", g.c);
    MDEMI_REQUIRE(g.kh > 0 && g.kw > 0 && g.stride > 0 && g.pad >= 0 && g.oh > 0 && g.ow > 0,
                  "gemm: bad conv geometry");
    const int64_t pixels = (int64_t)g.n * g.oh * g.ow;
    const int64_t taps = (int64_t)g.kh * g.kw * g.c;
    if (d->a_layout == MDEMI_L_CONV)
      MDEMI_REQUIRE(d->M == pixels && d->K == taps, "gemm: conv A needs M=N*OH*OW and K=KH*KW*C");
    if (d->b_layout == MDEMI_L_CONV)
      MDEMI_REQUIRE(d->K == pixels && d->N == taps && d->N % 4 == 0,
                    "gemm: conv B needs K=N*OH*OW and N=KH*KW*C");
    MDEMI_REQUIRE(al16(d->a_layout == MDEMI_L_CONV ? d->A : d->B), "gemm: conv operand must be 16-B aligned");
  }
  MDEMI_REQUIRE(d->bias_mode == MDEMI_BIAS_NONE || d->bias, "gemm: bias pointer missing");
  MDEMI_REQUIRE(d->act != MDEMI_ACT_GELU_GRAD || d->aux, "gemm: GELU-grad epilogue needs aux");
  return MDEMI_OK;
}

static void fill_params(const mdemi_gemm_desc* d, GemmParams& p) {
  p.M = d->M; p.N = d->N; p.K = d->K; p.batch = d->batch;
  p.A = d->A; p.lda = d->lda; p.a_bs = d->a_bstride;
  p.B = d->B; p.ldb = d->ldb; p.b_bs = d->b_bstride;
  p.C = d->C; p.ldc = d->ldc; p.c_bs = d->c_bstride;
  p.alpha = d->alpha; p.beta = d->beta;
  p.bias = d->bias; p.bias_mode = d->bias_mode; p.act = d->act;
  p.aux = d->aux; p.ldaux = d->ldaux; p.aux_bs = d->aux_bstride;
  p.res = d->residual; p.ldres = d->ldres; p.res_bs = d->res_bstride;
  p.cv = d->conv;
  const int ktiles = (int)cdiv(d->K, GBK);
  int split = d->split_k < ktiles ? d->split_k : ktiles;
  p.ktile_per_split = (int)cdiv(ktiles, split);
  p.split = (int)cdiv(ktiles, p.ktile_per_split);
  // vector loads need every row start 16-B aligned
  p.a_vec = al16(d->A) && (d->lda % 4 == 0) && (d->a_bstride % 4 == 0);
  p.b_vec = al16(d->B) && (d->ldb % 4 == 0) && (d->b_bstride % 4 == 0);
  p.slab = nullptr;
}

}  // namespace mdemi

using namespace mdemi;

extern "C" size_t mdemi_gemm_workspace_size(const mdemi_gemm_desc* d) {
  if (!d || d->split_k <= 1) return 0;
  GemmParams p;
  fill_params(d, p);
  if (p.split <= 1) return 0;
  return (size_t)p.split * d->batch * (size_t)d->M * d->N * sizeof(float);
}

extern "C" int mdemi_gemm_f32(const mdemi_gemm_desc* d, void* stream) {
  int rc = validate(d);
  if (rc) return rc;
  KernelFn fn = pick_kernel(d->a_layout, d->b_layout, d->a_op, d->b_op);
  if (!fn) {
    set_error("gemm: unsupported layout/op combination a=%d/%d b=%d/%d", d->a_layout, d->a_op, d->b_layout,
              d->b_op);
    return MDEMI_EUNSUP;
  }
  GemmParams p;
  fill_params(d, p);
  if (p.split > 1) {
    const size_t need = (size_t)p.split * d->batch * (size_t)d->M * d->N * sizeof(float);
    if (!d->workspace || (size_t)d->workspace_bytes < need) {
      set_error("gemm: split-K needs %zu workspace bytes", need);
      return MDEMI_EWORKSPACE;
    }
    p.slab = (float*)d->workspace;
  }
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)cdiv(d->N, GBN), (unsigned)cdiv(d->M, GBM), (unsigned)(d->batch * p.split));
  MDEMI_REQUIRE(grid.y <= 65535 && grid.z <= 65535, "gemm: grid too large");
  hipLaunchKernelGGL(fn, grid, dim3(GTHREADS), 0, st, p);
  if (p.split > 1) {
    const int64_t total = (int64_t)d->M * d->N * d->batch;
    const int nb = (int)(cdiv(total, 256) < 4096 ? cdiv(total, 256) : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(nb), dim3(256), 0, st, p);
  }
  return check_launch("gemm_f32");
}
