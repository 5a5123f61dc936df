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
// 64x64 = 2x2 MFMA 32x32 accumulators.  MFMA k-step s of a K tile takes, in
// lane half h, k = 8*(s/4) + 4*h + (s%4).  Both operands are staged in LDS as
// [k][row] images read with ds_read_b32 (32 consecutive floats per half-wave,
// conflict-free): M/N-contiguous sources are written as float4 rows (pitch
// 132), k-contiguous sources are transposed on the way in (4x ds_write_b32,
// pitch 130).  Register-staged prefetch of the next K tile (issue early, write
// late) into the second of two LDS buffers, one barrier per tile.  Block ids
// are remapped so that the tiles an XCD runs concurrently share A row-panels
// and B column-panels in that XCD's L2 (guide T1).  Variants: see pick_variant.
#include "common.h"
#include "gemm_core.h"
#include "gemm_f32_kernel.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace mdemi {

// Deterministic split-K combine + epilogue: sums slabs in split order.
// Deterministic split-K combine + epilogue: sums slabs in split order, four
// consecutive columns per thread when N % 4 == 0; also folds the row-sum
// partials [split][M] of a weight-gradient GEMM (bias gradient) in the same launch.
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemmParams p, const float* __restrict__ rs_part,
                                                          float* __restrict__ rs_out) {
  const int64_t MN = (int64_t)(p.M - p.m_split) * p.N;  // the split rows [m_split, M)
  const bool quad = (p.N & 3) == 0;
  const int64_t units = quad ? MN / 4 : MN;
  const int64_t total = units * p.batch;
  const int64_t slab_stride = (int64_t)p.batch * MN;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, gstride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = gid; e < total; e += gstride) {
    const int b = (int)(e / units);
    const int64_t u = e - (int64_t)b * units;
    const int64_t rem = quad ? 4 * u : u;
    const int i = (int)(rem / p.N) + p.m_split, j = (int)(rem - (int64_t)(i - p.m_split) * p.N);
    const float* src = p.slab + (int64_t)b * MN + rem;
    float* dst = p.C + boff(p, b, p.c_bs, p.c_bs2) + (int64_t)i * p.ldc + j;
    __bf16* dst16 = p.c16 ? reinterpret_cast<__bf16*>(p.c16) + (dst - p.C) : nullptr;  // C's layout
    if (quad) {
      float4 acc = *reinterpret_cast<const float4*>(src);
      for (int q = 1; q < p.split; ++q) {
        const float4 t = *reinterpret_cast<const float4*>(src + q * slab_stride);
        acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
      }
      const float v[4] = {epilogue_value(p, b, i, j, acc.x), epilogue_value(p, b, i, j + 1, acc.y),
                          epilogue_value(p, b, i, j + 2, acc.z), epilogue_value(p, b, i, j + 3, acc.w)};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dst[e] = v[e];
        if (dst16) dst16[e] = (__bf16)v[e];
      }
    } else {
      float acc = src[0];
      for (int q = 1; q < p.split; ++q) acc += src[q * slab_stride];
      const float v = epilogue_value(p, b, i, j, acc);
      dst[0] = v;
      if (dst16) dst16[0] = (__bf16)v;
    }
  }
  if (rs_part)
    for (int64_t i = gid; i < p.M; i += gstride) {
      float acc = rs_part[i];
      for (int q = 1; q < p.split; ++q) acc += rs_part[(int64_t)q * p.M + i];
      rs_out[i] = acc;
    }
}


// Variants (tools/gemm_bench.py on the NewCRFs-L07 480x640 bs=8 shapes,
// profiles/r01_gemm_variants_v2.log):
//   0: BK16, 2 LDS buffers, register prefetch, k-contiguous operands transposed
//      into [k][row] images (ds_read_b32 fragments)
//   1: as 0 with [row][k] images (ds_read_b128 fragments)
//   2: as 0 capped at 128 VGPRs (4 waves/SIMD; spills)
//   3: BK32, 2 buffers (2 workgroups/CU by LDS)   4: BK32, 1 buffer   5: as 3, [row][k]
//   6: 256-row tile (waves of 128x64), BK32, 1 buffer   7: 256-row tile, BK16, 2 buffers
//   (a BK64 single-buffer variant measured no faster than 4 on the model's shapes:
//   profiles/round3/gemm_study_bk64.txt)
//   8..12: direct-to-LDS staging (buffer_load ... lds, gemm_glds_kernel.h), dense 16-B
//   operands without a load-time op only: 8 128-row BK32, 9 256-row BK16, 10 256-row
//   BK32 (96 KiB, one workgroup per CU), 11 128-row BK16, 12 128-row x 192-column BK32 (the
//   N = 192 / 576 shapes of the Swin stage 0: no half-empty 128-column tile)
// No variant wins every shape (e.g. weight-gradient GEMMs over few output
// tiles want BK32/2 buffers, token-major forwards want BK32/1 buffer), so by
// default each distinct (layouts, ops, M, N, K, batch, split) is timed once
// over the candidates on first use and the winner cached.  All variants add
// the k products in the same order and split K at the same 32-element
// boundaries, so the choice never changes a result bit.
constexpr int NVARIANTS = 13;
static int g_variant = -1;  // -1: autotune per shape
// A/B switches (environment, read once): MDEMI_GEMM_TAIL_SPLIT=0 disables the tail split;
// MDEMI_GEMM_INLINE_REDUCE=1 (fp32) / MDEMI_GEMM_INLINE_REDUCE_B16=1 (bf16) combine split-K
// slabs in the kernel (the tile's last-arriving workgroup) instead of the separate reduce
// kernel.  The separate, chip-wide reduce is the default since round 6: one last arriver
// reading every other slab of its tile serialises on a workgroup's fetch rate (~32 GB/s:
// profiles/round6/b16_variants_*.txt), which the bf16 step's small-grid weight gradients
// hit hardest -- configs[4] 145.5 -> 152.2 img/s, NYU 60.2 -> 60.8, AdaBins 73.6 -> 73.9 on
// one box (profiles/round6/ab_inline_reduce.txt).  The tail split always combines inline.
static bool env_on(const char* name) {
  const char* v = getenv(name);
  return !(v && v[0] == '0');
}
static bool env_set(const char* name) {
  const char* v = getenv(name);
  return v && v[0] && v[0] != '0';
}
static bool g_tail_split = env_on("MDEMI_GEMM_TAIL_SPLIT");
static bool g_inline_reduce = env_set("MDEMI_GEMM_INLINE_REDUCE");
static bool g_inline_reduce_b16 = env_set("MDEMI_GEMM_INLINE_REDUCE_B16");
static int g_variant_m16 = -1;  // 16-bit family (bf16 / split fp32): 0 two LDS buffers, 1 one
static int g_variant_b16 = -1;  // bf16-operand family: 0 128-row tile, 1 256-row tile, 2 128-row x 2 K tiles
static int g_group_m = 8;

KernelFn f32_pick_part0(int al, int bl, int aop, int bop, int v);
KernelFn f32_pick_part1(int al, int bl, int aop, int bop, int v);
KernelFn f32_pick_part2(int al, int bl, int aop, int bop, int v);
KernelFn f32_pick_part3(int al, int bl, int aop, int bop, int v);

KernelFn glds_pick_part0(int al, int bl, int v);
KernelFn glds_pick_part1(int al, int bl, int v);

static KernelFn pick_kernel(int al, int bl, int aop, int bop, int v) {
  if (v >= 8) {  // direct-to-LDS variants: dense operands without a load-time op
    if (aop != MDEMI_OP_NONE || bop != MDEMI_OP_NONE) return nullptr;
    if (KernelFn f = glds_pick_part0(al, bl, v)) return f;
    return glds_pick_part1(al, bl, v);
  }
  if (KernelFn f = f32_pick_part0(al, bl, aop, bop, v)) return f;
  if (KernelFn f = f32_pick_part1(al, bl, aop, bop, v)) return f;
  if (KernelFn f = f32_pick_part2(al, bl, aop, bop, v)) return f;
  return f32_pick_part3(al, bl, aop, bop, v);
}

static int variant_bk(int v, int mode) {
  if (mode != GEMM_F32) return 32;  // the 16-bit and bf16-operand families: BK 32
  if (v >= 8) return (v == 8 || v == 10 || v == 12) ? 32 : 16;
  return (v >= 3 && v != 7) ? 32 : 16;
}
static int variant_cols(int v, int mode) { return (mode == GEMM_F32 && v == 12) ? 192 : GBN; }
static int variant_rows(int v, int mode) {
  if (mode == GEMM_B16) return v == 1 ? 2 * GBM : GBM;
  return (mode != GEMM_F32 ? (v == 2 || v == 4) : (v == 6 || v == 7 || v == 9 || v == 10)) ? 2 * GBM : GBM;
}
// the direct-to-LDS variants need dense operands that load as whole 16-B quads and no
// load-time transform
static bool glds_ok(const mdemi_gemm_desc* d, const GemmParams& p) {
  return d->a_layout != MDEMI_L_CONV && d->b_layout != MDEMI_L_CONV && d->a_op == MDEMI_OP_NONE &&
         d->b_op == MDEMI_OP_NONE && p.a_vec && p.b_vec;
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
    MDEMI_REQUIRE(g.kh > 0 && g.kw > 0 && g.stride > 0 && g.pad > -1024 && g.oh > 0 && g.ow > 0,
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
  MDEMI_REQUIRE(!d->rowsum_a || (d->a_layout == MDEMI_L_MNCONTIG && d->batch == 1),
                "gemm: rowsum_a needs an m-contiguous A and batch 1");
  if (d->rowsum_a) MDEMI_REQUIRE(d->rowsum_a != d->C, "gemm: rowsum_a must not alias C");
  if (d->row_scale)
    MDEMI_REQUIRE(d->batch == 1 && d->row_scale_group > 0 && d->row_scale_group < ((int64_t)1 << 31),
                  "gemm: row_scale needs batch 1 and 0 < row_scale_group < 2^31");
  if (d->batch_inner > 1)
    MDEMI_REQUIRE(d->batch % d->batch_inner == 0 && !d->aux && !d->residual && !d->preact && !d->rowsum_a,
                  "gemm: batch_inner needs batch %% batch_inner == 0 and no aux/residual/preact/rowsum_a");
  // tile-relative 32-bit buffer offsets: 128 rows (or 16 k-rows) of any leading dimension
  const int64_t lim = (int64_t)1 << 21;
  MDEMI_REQUIRE(d->lda < lim && d->ldb < lim && d->ldc < lim && d->ldaux < lim && d->ldres < lim &&
                    d->ldpre < lim, "gemm: leading dimension too large for 32-bit tile offsets");
  if (d->split_k > 1)
    MDEMI_REQUIRE(d->N < lim, "gemm: N too large for split-K slabs");
  MDEMI_REQUIRE(!(d->act == MDEMI_ACT_GELU_GRAD || d->act == MDEMI_ACT_RELU_GRAD || d->act == MDEMI_ACT_SILU_GRAD) ||
                    d->aux, "gemm: *_GRAD epilogue needs aux");
  return MDEMI_OK;
}

static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    hipDeviceProp_t pr;
    cus[dev] = hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0 ? pr.multiProcessorCount
                                                                                           : 256;
  }
  return cus[dev];
}

// Tail split.  A whole-K GEMM whose 128x128 tiles fill R full rounds of resident
// workgroups plus a thin last round (profiles/round3: 9600x3072x768 = 2.34 rounds of the
// 3-workgroup/CU variant runs at 115 TF/s vs 130 at exactly 2 or 3 rounds) splits the rows
// holding the leftover tiles into `split` K pieces, which fit in the last round's free
// slots, and the last-arriving piece of each tile combines them.  The plan depends on the
// shape only (rows cut at a 256-row boundary, K at the family's 32-element chunks), so every
// variant splits the same outputs the same way and the family stays bit-identical.
struct TailPlan {
  int m_split, split;  // split 1: no tail split
};
static TailPlan tail_plan(const mdemi_gemm_desc* d) {
  TailPlan t{0, 1};
  if (!g_tail_split || d->split_k > 1 || d->batch != 1 || d->rowsum_a) return t;
  const int64_t tm = cdiv(d->M, 128), tn = cdiv(d->N, 128), T = tm * tn;
  const int64_t S = 3LL * device_cus();  // resident 128x128 tiles (3 workgroups per CU)
  const int64_t full = T / S, rem = T - full * S;
  if (full < 1 || rem == 0 || rem * 10 > S * 6) return t;  // no thin last round
  const int64_t m_split = (tm - cdiv(rem, tn)) / 2 * 256;
  if (m_split <= 0) return t;
  const int64_t tail_tiles = cdiv(d->M - m_split, 128) * tn;
  int64_t s = std::min<int64_t>(4, S / tail_tiles);
  s = std::min<int64_t>(s, cdiv(d->K, 32) / 2);  // every piece keeps >= 2 K chunks
  if (s < 2) return t;
  t.m_split = (int)m_split;
  t.split = (int)s;
  return t;
}

static void fill_params(const mdemi_gemm_desc* d, GemmParams& p, int variant, int mode) {
  const int GBK = variant_bk(variant, mode);
  p.M = d->M; p.N = d->N; p.K = d->K; p.batch = d->batch;
  p.A = d->A; p.lda = d->lda; p.a_bs = d->a_bstride;
  p.B = d->B; p.ldb = d->ldb; p.b_bs = d->b_bstride;
  p.C = d->C; p.ldc = d->ldc; p.c_bs = d->c_bstride;
  p.alpha = d->alpha; p.beta = d->beta;
  p.bias = d->bias; p.bias_mode = d->bias_mode; p.act = d->act;
  p.aux = d->aux; p.ldaux = d->ldaux; p.aux_bs = d->aux_bstride;
  p.res = d->residual; p.ldres = d->ldres; p.res_bs = d->res_bstride;
  p.cv = d->conv;
  p.pre = d->preact; p.ldpre = d->ldpre; p.pre_bs = d->pre_bstride;
  p.rowsum = d->rowsum_a;
  p.rowscale = d->row_scale;
  if (d->row_scale) p.fd_rs = make_fastdiv((uint32_t)d->row_scale_group);
  p.binner = d->batch_inner > 1 ? d->batch_inner : 1;
  p.a_bs2 = p.binner > 1 ? d->a_bstride_inner : 0;
  p.b_bs2 = p.binner > 1 ? d->b_bstride_inner : 0;
  p.c_bs2 = p.binner > 1 ? d->c_bstride_inner : 0;
  // split boundaries in fixed 32-element K chunks whatever the variant's BK, so the
  // variants of a family agree bit for bit
  const int CH = 32;
  const int kc = (int)cdiv(d->K, CH);
  const TailPlan tp = tail_plan(d);
  const int want = tp.split > 1 ? tp.split : d->split_k;
  const int split = want < kc ? want : kc;
  const int chunks_per_split = (int)cdiv(kc, split);
  p.ktile_per_split = chunks_per_split * (CH / GBK);
  p.split = (int)cdiv(kc, chunks_per_split);
  p.m_split = (tp.split > 1 && p.split > 1) ? tp.m_split : 0;
  p.tile_cnt = nullptr;
  p.rowsum_out = nullptr;
  p.c16 = nullptr;
  // vector loads need every row start 16-B aligned and whole quads in range
  // (KCONTIG: K % 4; MNCONTIG: the row/column extent % 4)
  p.a_vec = al16(d->A) && (d->lda % 4 == 0) && (d->a_bstride % 4 == 0) && (p.a_bs2 % 4 == 0) &&
            (d->a_layout == MDEMI_L_KCONTIG ? d->K % 4 == 0 : d->M % 4 == 0);
  p.b_vec = al16(d->B) && (d->ldb % 4 == 0) && (d->b_bstride % 4 == 0) && (p.b_bs2 % 4 == 0) &&
            (d->b_layout == MDEMI_L_KCONTIG ? d->K % 4 == 0 : d->N % 4 == 0);
  if (d->a_layout == MDEMI_L_CONV || d->b_layout == MDEMI_L_CONV) {
    const mdemi_conv_geom& g = d->conv;
    p.fd_c = make_fastdiv(g.c); p.fd_kw = make_fastdiv(g.kw);
    p.fd_ow = make_fastdiv(g.ow); p.fd_oh = make_fastdiv(g.oh);
  }
  p.slab = nullptr;
  const int vrows = variant_rows(variant, mode);  // 256-row variants: 16-bit 2, fp32 6 and 7
  p.tiles_m1 = p.m_split / vrows;
  p.tiles_m = (int)cdiv(d->M - p.m_split, vrows);
  p.tiles_n = (int)cdiv(d->N, variant_cols(variant, mode));
  p.group_m = g_group_m;
}

}  // namespace mdemi

using namespace mdemi;

static size_t slab_bytes(const mdemi_gemm_desc* d, const GemmParams& p) {
  return p.split > 1 ? align_up((size_t)p.split * d->batch * (size_t)(d->M - p.m_split) * d->N * sizeof(float), 256)
                     : 0;
}

// Per-device split-tile counters for the in-kernel slab combine: zeroed once on the
// launch stream, left zeroed by every launch (the last arriver resets its tile's slot).
// GEMMs with split tiles on two streams at once would share them: the library runs its
// GEMMs on one compute stream.  None is allocated during a graph capture (nullptr: the
// launch falls back to the reduce kernel); a grown buffer keeps the old one alive for
// graphs that recorded it.
static int* tile_counters(int64_t n, hipStream_t st) {
  static std::mutex mu;
  static std::map<int, std::pair<int*, int64_t>> bufs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto& e = bufs[dev];
  if (e.second >= n) return e.first;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  const int64_t cap = std::max<int64_t>(n, (int64_t)1 << 16);
  int* ptr = nullptr;
  if (hipMalloc(&ptr, cap * sizeof(int)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(ptr, 0, cap * sizeof(int), st) != hipSuccess) return nullptr;
  e = {ptr, cap};
  return ptr;
}
static size_t rowsum_bytes(const mdemi_gemm_desc* d, const GemmParams& p) {
  return (p.split > 1 && d->rowsum_a) ? (size_t)p.split * d->M * sizeof(float) : 0;
}

// split-K combine by column sums: deep splits with a plain store epilogue
static bool colsum_combine(const mdemi_gemm_desc* d, const GemmParams& p) {
  return p.split >= 32 && d->batch == 1 && d->alpha == 1.f && d->beta == 0.f && d->bias_mode == MDEMI_BIAS_NONE &&
         d->act == MDEMI_ACT_NONE && !d->residual && !d->preact && d->ldc == d->N;
}
static size_t colsum_combine_bytes(const mdemi_gemm_desc* d, const GemmParams& p) {
  return colsum_combine(d, p) ? colsum_ws_bytes(p.split, (int64_t)d->M * d->N) : 0;
}

// bf16 operands / output of mdemi_gemm_bf16x (null for the fp32-operand entry points)
struct B16Ext {
  const void* a16; const void* b16; void* c16;
};

static int launch(const mdemi_gemm_desc* d, int variant, hipStream_t st, int mode, const B16Ext* ext = nullptr) {
  if (mode == GEMM_F32E && variant >= 3) variant = 0;  // the bf16-image variants hold one bf16 plane
  if (mode == GEMM_F32 && variant >= 8) {  // a forced direct-to-LDS variant on an operand it cannot stage
    GemmParams q;
    fill_params(d, q, variant, mode);
    if (!glds_ok(d, q)) variant = 0;
  }
  KernelFn fn = mode == GEMM_F32   ? pick_kernel(d->a_layout, d->b_layout, d->a_op, d->b_op, variant)
                : mode == GEMM_B16 ? pick_kernel_b16(d->a_layout, d->b_layout, variant)
                                   : pick_kernel_m16(d->a_layout, d->b_layout, d->a_op, d->b_op,
                                                     mode == GEMM_BF16 ? 1 : 3, variant);
  if (!fn) {
    set_error("gemm: unsupported layout/op combination a=%d/%d b=%d/%d", d->a_layout, d->a_op, d->b_layout,
              d->b_op);
    return MDEMI_EUNSUP;
  }
  GemmParams p;
  fill_params(d, p, variant, mode);
  if (ext) {
    p.c16 = ext->c16;
    if (mode == GEMM_B16) {  // the kernel reads the bf16 tensors through the A/B slots
      p.A = reinterpret_cast<const float*>(ext->a16);
      p.B = reinterpret_cast<const float*>(ext->b16);
    }
  }
  float* rowsum_part = nullptr;
  if (p.split > 1) {
    const size_t need = slab_bytes(d, p) + rowsum_bytes(d, p) + colsum_combine_bytes(d, p);
    if (!d->workspace || (size_t)d->workspace_bytes < need) {
      set_error("gemm: split-K needs %zu workspace bytes", need);
      return MDEMI_EWORKSPACE;
    }
    p.slab = (float*)d->workspace;
    if (d->rowsum_a) {
      rowsum_part = (float*)((char*)d->workspace + slab_bytes(d, p));
      p.rowsum = rowsum_part;
    }
  }
  const int64_t nblocks = (int64_t)p.tiles_m1 * p.tiles_n + (int64_t)p.tiles_m * p.tiles_n * d->batch * p.split;
  MDEMI_REQUIRE(nblocks < (int64_t)1 << 31, "gemm: grid too large");
  const bool deep = p.split > 1 && colsum_combine(d, p) && !p.c16;  // the column-sum combine writes fp32 only
  // both bf16 families (bf16 operands in HBM, or rounded at staging) combine alike, so the
  // bf16-storage step stays bit-identical to the fp32-operand bf16 step
  const bool inline_reduce = (mode == GEMM_B16 || mode == GEMM_BF16) ? g_inline_reduce_b16 : g_inline_reduce;
  if (p.split > 1 && !deep && (inline_reduce || p.m_split > 0)) {
    p.tile_cnt = tile_counters((int64_t)p.tiles_m * p.tiles_n * d->batch, st);
    if (p.tile_cnt && rowsum_part) p.rowsum_out = d->rowsum_a;  // the last arrivers sum the row partials
  }
  hipLaunchKernelGGL(fn, dim3((unsigned)nblocks), dim3(GTHREADS), 0, st, p);
  if (p.split > 1 && !p.tile_cnt) {
    if (deep) {
      // many slabs over a small C (skinny weight gradients over ~10^6 pixels): a
      // column sum parallel over the slab rows, not one thread per output summing
      // `split` dependent loads
      char* cws = (char*)d->workspace + slab_bytes(d, p) + rowsum_bytes(d, p);
      int rc = colsum_launch(p.slab, p.split, (int64_t)d->M * d->N, (int64_t)d->M * d->N, d->C, 0, cws, st);
      if (!rc && rowsum_part) rc = colsum_launch(rowsum_part, p.split, d->M, d->M, d->rowsum_a, 0, cws, st);
      if (rc) return rc;
    } else {
      const int64_t total = (int64_t)(d->M - p.m_split) * d->N * d->batch / ((d->N & 3) == 0 ? 4 : 1);
      const int nb = (int)(cdiv(total, 256) < 4096 ? cdiv(total, 256) : 4096);
      hipLaunchKernelGGL(gemm_splitk_reduce, dim3(nb), dim3(256), 0, st, p, (const float*)rowsum_part,
                         rowsum_part ? d->rowsum_a : (float*)nullptr);
    }
  }
  return check_launch(mode == GEMM_BF16 ? "gemm_bf16" : mode == GEMM_F32E ? "gemm_f32e" : mode == GEMM_B16 ? "gemm_bf16x" : "gemm_f32");
}

struct TuneKey {
  int al, bl, aop, bop, M, N, K, batch, split, mode;
  bool operator<(const TuneKey& o) const {
    return std::tie(al, bl, aop, bop, M, N, K, batch, split, mode) <
           std::tie(o.al, o.bl, o.aop, o.bop, o.M, o.N, o.K, o.batch, o.split, o.mode);
  }
};
static std::map<TuneKey, int> g_tuned;
static std::mutex g_tune_mu;

// Re-running the GEMM is only harmless when C is write-only and aliases no input.
static bool tunable(const mdemi_gemm_desc* d, hipStream_t st) {
  if (d->beta != 0.f) return false;
  const void* c = d->C;
  if (c == d->A || c == d->B || c == d->residual || c == d->aux || c == d->bias) return false;
  if (d->rowsum_a && (d->rowsum_a == d->A || d->rowsum_a == d->B)) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
  return true;
}

static int choose_variant(const mdemi_gemm_desc* d, hipStream_t st, int mode, const B16Ext* ext = nullptr) {
  if (mode == GEMM_B16) {
    if (g_variant_b16 >= 0) return g_variant_b16;
  } else if (mode != GEMM_F32 ? g_variant_m16 >= 0 : g_variant >= 0) {
    return mode != GEMM_F32 ? g_variant_m16 : g_variant;
  }
  const TuneKey key{d->a_layout, d->b_layout, d->a_op, d->b_op, d->M, d->N, d->K, d->batch, d->split_k, mode};
  {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    auto it = g_tuned.find(key);
    if (it != g_tuned.end()) return it->second;
  }
  if (!tunable(d, st)) return 0;
  if (ext && ext->c16 && (ext->c16 == ext->a16 || ext->c16 == ext->b16)) return 0;
  static const int cands_f32[] = {0, 1, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12};
  static const int cands_m16[] = {0, 1, 2, 3, 4};
  const int* cands = mode != GEMM_F32 ? cands_m16 : cands_f32;
  int ncand = mode == GEMM_BF16 ? 5 : mode == GEMM_F32E ? 3 : mode == GEMM_B16 ? 3 : 12;
  if (mode == GEMM_F32) {
    GemmParams q;
    fill_params(d, q, 0, mode);
    if (!glds_ok(d, q)) ncand = 7;
  }
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 0;
  int best = 0;
  float best_ms = 1e30f;
  for (int ci = 0; ci < ncand; ++ci) {
    const int v = cands[ci];
    if (launch(d, v, st, mode, ext) != MDEMI_OK) continue;  // warm (and validate)
    (void)hipEventRecord(e0, st);
    for (int r = 0; r < 3; ++r) launch(d, v, st, mode, ext);
    (void)hipEventRecord(e1, st);
    float ms = 0.f;
    if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) continue;
    if (ms < best_ms) { best_ms = ms; best = v; }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  std::lock_guard<std::mutex> lk(g_tune_mu);
  g_tuned[key] = best;
  return best;
}

extern "C" size_t mdemi_gemm_workspace_size(const mdemi_gemm_desc* d) {
  if (!d) return 0;
  GemmParams p;
  fill_params(d, p, 0, GEMM_F32);  // every family splits at the same 32-element chunks
  if (p.split <= 1) return 0;
  return slab_bytes(d, p) + rowsum_bytes(d, p) + colsum_combine_bytes(d, p);
}

static int gemm_entry(const mdemi_gemm_desc* d, void* stream, int mode) {
  int rc = validate(d);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  return launch(d, choose_variant(d, st, mode), st, mode);
}

// bf16-operand path: both operands bf16 in HBM and a layout the DMA loaders stage (16-B
// quads of 8 bf16: k-contiguous K % 8, m/n-contiguous extent % 8, implicit-im2col C % 8,
// leading dimensions and batch strides % 8, 16-B aligned bases, no load-time op, no
// bias-gradient row sums -- those are summed from the unrounded fp32 operand)
static bool al16v(const void* p) { return ((uintptr_t)p & 15) == 0; }
static bool b16_ok(const mdemi_gemm_desc* d, const B16Ext& e) {
  if (!e.a16 || !e.b16 || !al16v(e.a16) || !al16v(e.b16)) return false;
  if (d->a_op != MDEMI_OP_NONE || d->b_op != MDEMI_OP_NONE || d->rowsum_a) return false;
  if (d->a_layout == MDEMI_L_CONV && d->b_layout == MDEMI_L_CONV) return false;
  auto operand = [&](int layout, int64_t ld, int64_t bs, int64_t bs2, int64_t extent) {
    if (layout == MDEMI_L_CONV) {
      const mdemi_conv_geom& g = d->conv;
      return g.c % 8 == 0 && (int64_t)g.n * g.h * g.w * g.c * 2 < ((int64_t)1 << 31);
    }
    if (ld % 8 || bs % 8 || bs2 % 8) return false;
    return layout == MDEMI_L_KCONTIG ? d->K % 8 == 0 : extent % 8 == 0;
  };
  const int64_t ai = d->batch_inner > 1 ? d->a_bstride_inner : 0, bi = d->batch_inner > 1 ? d->b_bstride_inner : 0;
  return operand(d->a_layout, d->lda, d->a_bstride, ai, d->M) && operand(d->b_layout, d->ldb, d->b_bstride, bi, d->N);
}

extern "C" int mdemi_gemm_bf16x(const mdemi_gemm_desc* d, const void* a16, const void* b16, void* c16, void* stream) {
  MDEMI_REQUIRE(d, "gemm: null descriptor");
  const B16Ext e{a16, b16, c16};
  hipStream_t st = (hipStream_t)stream;
  if (b16_ok(d, e)) {
    mdemi_gemm_desc v = *d;  // validate() checks the fp32 operand slots; the bf16 ones stand in
    v.A = (const float*)a16;
    v.B = (const float*)b16;
    int rc = validate(&v);
    if (rc) return rc;
    return launch(d, choose_variant(d, st, GEMM_B16, &e), st, GEMM_B16, &e);
  }
  // a layout the bf16 loaders cannot stage: the m16 family on the fp32 operands (the same
  // bf16 products, bit for bit)
  MDEMI_REQUIRE(d->A && d->B, "gemm_bf16x: no bf16 path for this layout (a=%d b=%d) and no fp32 operands given",
                d->a_layout, d->b_layout);
  int rc = validate(d);
  if (rc) return rc;
  const B16Ext f{nullptr, nullptr, c16};
  return launch(d, choose_variant(d, st, GEMM_BF16, &f), st, GEMM_BF16, &f);
}

extern "C" int mdemi_gemm_bf16x_supported(const mdemi_gemm_desc* d, const void* a16, const void* b16) {
  return d && b16_ok(d, B16Ext{a16, b16, nullptr}) ? 1 : 0;
}

extern "C" int mdemi_gemm_f32(const mdemi_gemm_desc* d, void* stream) { return gemm_entry(d, stream, GEMM_F32); }
extern "C" int mdemi_gemm_bf16(const mdemi_gemm_desc* d, void* stream) { return gemm_entry(d, stream, GEMM_BF16); }
extern "C" int mdemi_gemm_f32e(const mdemi_gemm_desc* d, void* stream) { return gemm_entry(d, stream, GEMM_F32E); }

// Benchmark/tuning hook: force a pipelining variant of the fp32 family (see
// pick_variant) and of the 16-bit family (gemm_mfma16.hip m16_variant; -1 =
// per-shape autotune, the default) and the tile raster (group_m > 0: XCD-aware
// grouped raster; 0: plain).
extern "C" int mdemi_gemm_set_variant(int32_t variant, int32_t group_m) {
  MDEMI_REQUIRE(variant >= -1 && variant < NVARIANTS && group_m >= 0, "gemm_set_variant: bad args");
  g_variant = variant;
  g_group_m = group_m;
  return MDEMI_OK;
}

extern "C" int mdemi_gemm_set_options(int32_t tail_split, int32_t inline_reduce) {
  g_tail_split = tail_split != 0;
  g_inline_reduce = inline_reduce != 0;
  return MDEMI_OK;
}

extern "C" int mdemi_gemm_set_variant_m16(int32_t variant) {
  MDEMI_REQUIRE(variant >= -1 && variant < 5, "gemm_set_variant_m16: bad variant");
  g_variant_m16 = variant;
  return MDEMI_OK;
}

extern "C" int mdemi_gemm_set_variant_b16(int32_t variant) {
  MDEMI_REQUIRE(variant >= -1 && variant < 3, "gemm_set_variant_b16: bad variant");
  g_variant_b16 = variant;
  return MDEMI_OK;
}
