// Elementwise sweeps, bias-gradient column sums, and the multi-tensor AdamW
// step with the global-norm clip folded in (restated train step: the
// reference's run.py/optimizer construction is absent; config keys
// optimizer.lr/weight_decay/betas/eps and train.grad_norm, e.g.
// json/nyu/newcrfs/newcrfs_github_eval.json).
#include <algorithm>

#include "common.h"

namespace mdemi {

__global__ __launch_bounds__(256) void ew_kernel(int op, const float* __restrict__ a, const float* __restrict__ b,
                                                 float* __restrict__ y, int64_t n, float s, float t) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float v;
    switch (op) {
      case MDEMI_EW_ADD: v = a[i] + b[i]; break;
      case MDEMI_EW_SIGMOID_SCALE: v = sigmoid_f(a[i]) * s; break;
      case MDEMI_EW_SIGMOID_SCALE_BWD: {
        const float sg = sigmoid_f(a[i]);
        v = b[i] * s * sg * (1.f - sg);
        break;
      }
      case MDEMI_EW_AXPBY: v = s * a[i] + t * b[i]; break;
      case MDEMI_EW_ACT_BWD: {
        const int act = (int)s;
        const float x = a[i];
        v = b[i] * act_grad(act, x, apply_act(act, x));
        break;
      }
      default: v = 0.f;
    }
    y[i] = v;
  }
}

// column sums: block (32 cols x 8 row-groups) partials over a row chunk
__global__ __launch_bounds__(256) void colsum_partial(const float* __restrict__ x, int64_t rows, int64_t cols,
                                                      int64_t ld, float* __restrict__ part, int64_t rows_per_blk) {
  __shared__ float red[8][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t c = (int64_t)blockIdx.x * 32 + tx;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_blk;
  const int64_t r1 = min(rows, r0 + rows_per_blk);
  float s = 0.f;
  if (c < cols)
    for (int64_t r = r0 + ty; r < r1; r += 8) s += x[r * ld + c];
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][tx];
    part[(int64_t)blockIdx.y * cols + c] = t;
  }
}

__global__ void colsum_final(const float* __restrict__ part, int nblk, int64_t cols, float* __restrict__ out,
                             float* __restrict__ out2, int64_t split_col, int accumulate) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int i = 0; i < nblk; ++i) s += part[(int64_t)i * cols + c];
  float* o = c < split_col ? out + c : out2 + (c - split_col);
  *o = accumulate ? *o + s : s;
}

// Short reductions (rows <= COLSUM_ONEPASS): one launch, no workspace.  A block
// covers 32 columns with 32 row groups; each thread issues all its (<= 32) loads at
// once -- one memory round trip instead of four -- and adds them in row order (rows
// ty, ty+32, ...), then the 32 group sums are added in group order: a fixed
// association, so the result is deterministic.
constexpr int COLSUM_ONEPASS = 1024;
__global__ __launch_bounds__(1024) void colsum_onepass(const float* __restrict__ x, int64_t rows, int64_t cols,
                                                       int64_t ld, float* __restrict__ out, float* __restrict__ out2,
                                                       int64_t split_col, int accumulate) {
  __shared__ float red[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t c = (int64_t)blockIdx.x * 32 + tx;
  float s = 0.f;
  if (c < cols) {
    constexpr int NL = COLSUM_ONEPASS / 32;
    float v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int64_t r = ty + 32 * j;
      v[j] = r < rows ? x[r * ld + c] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) s += v[j];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) t += red[k][tx];
    float* o = c < split_col ? out + c : out2 + (c - split_col);
    *o = accumulate ? *o + t : t;
  }
}

static int colsum_blocks_y(int64_t rows) {
  int64_t ny = cdiv(rows, 512);
  return (int)(ny < 256 ? (ny < 1 ? 1 : ny) : 256);
}

// ---------------- optimizer ----------------
constexpr int OPT_THREADS = 256;
constexpr int OPT_CHUNK = 65536;  // elements per (tensor, chunk) work item

struct AdamGroups {
  mdemi_adamw_group g[4];
};

// gradients as the update sees them: g * gs (gs = 1/world when the data-parallel mean's
// scale is folded in here instead of a sweep over the reduced gradients; 1 otherwise)
__device__ __forceinline__ float4 scale4(float4 g, float gs) {
  if (gs != 1.f) { g.x *= gs; g.y *= gs; g.z *= gs; g.w *= gs; }
  return g;
}

// per-tensor sum of squares partials: one block per (tensor, chunk); float4
// loads over the 16-B-aligned body of the chunk (torch allocations are 256-B
// aligned and chunks are multiples of 4 elements), scalar tail
__global__ __launch_bounds__(OPT_THREADS) void sumsq_partial(const mdemi_tensor_ref* __restrict__ tl, int nt,
                                                             const int* __restrict__ chunk_tensor,
                                                             const int* __restrict__ chunk_index,
                                                             float* __restrict__ part, float gs) {
  __shared__ float red[OPT_THREADS / 64];
  const int item = blockIdx.x;
  const mdemi_tensor_ref t = tl[chunk_tensor[item]];
  const int64_t beg = (int64_t)chunk_index[item] * OPT_CHUNK;
  const int64_t end = min(t.numel, beg + OPT_CHUNK);
  // four independent float4 streams per thread keep 4 loads in flight and 4 FMA chains
  float s4[4] = {0.f, 0.f, 0.f, 0.f};
  const bool vec = ((uintptr_t)t.grad & 15) == 0;
  const int64_t vend = vec ? beg + ((end - beg) & ~(int64_t)3) : beg;
  constexpr int64_t STEP = 4 * OPT_THREADS;
  int64_t i = beg + 4 * threadIdx.x;
  for (; i + 3 * STEP < vend; i += 4 * STEP) {
    float4 g[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) g[u] = scale4(*reinterpret_cast<const float4*>(t.grad + i + u * STEP), gs);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s4[u] = fmaf(g[u].x, g[u].x, s4[u]); s4[u] = fmaf(g[u].y, g[u].y, s4[u]);
      s4[u] = fmaf(g[u].z, g[u].z, s4[u]); s4[u] = fmaf(g[u].w, g[u].w, s4[u]);
    }
  }
  for (; i < vend; i += STEP) {
    const float4 g = scale4(*reinterpret_cast<const float4*>(t.grad + i), gs);
    s4[0] = fmaf(g.x, g.x, s4[0]); s4[0] = fmaf(g.y, g.y, s4[0]);
    s4[0] = fmaf(g.z, g.z, s4[0]); s4[0] = fmaf(g.w, g.w, s4[0]);
  }
  for (int64_t j = vend + threadIdx.x; j < end; j += OPT_THREADS) {
    const float g = gs != 1.f ? t.grad[j] * gs : t.grad[j];
    s4[1] = fmaf(g, g, s4[1]);
  }
  float s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  s = block_sum<OPT_THREADS>(s, red);
  if (threadIdx.x == 0) part[item] = s;
}

__global__ void sumsq_final(const float* __restrict__ part, int nitems, float* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nitems; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)red[0];
}

// torch.optim.AdamW on one (tensor, chunk) item (decoupled weight decay,
// non-amsgrad, foreach=False semantics); `step` is the 1-based step count
// p16 (optional): also write the RNE bf16 copy of the updated parameter -- the operand
// its bf16 GEMMs read next step (what mdemi_cast_bf16 would produce, bit for bit)
typedef __bf16 opt_bf16x4_t __attribute__((ext_vector_type(4)));
typedef float opt_f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void adamw_item(const mdemi_tensor_ref& t, const mdemi_adamw_group& gp, float clip,
                                           float gs, float step, int64_t beg, int64_t end,
                                           __bf16* __restrict__ p16 = nullptr) {
  const float b1 = gp.beta1, b2 = gp.beta2;
  const float step_size = gp.lr / (1.f - powf(b1, step));
  const float bc2s = sqrtf(1.f - powf(b2, step));
  const float decay = 1.f - gp.lr * gp.weight_decay;
  auto upd = [&](float g, float& p, float& m, float& v) {
    if (gs != 1.f) g *= gs;
    g *= clip;
    p *= decay;
    m = m * b1 + (1.f - b1) * g;
    v = v * b2 + (1.f - b2) * g * g;
    p -= step_size * m / (sqrtf(v) / bc2s + gp.eps);
  };
  const bool vec = (((uintptr_t)t.param | (uintptr_t)t.grad | (uintptr_t)t.exp_avg | (uintptr_t)t.exp_avg_sq) & 15) == 0 &&
                   ((uintptr_t)p16 & 7) == 0;
  const int64_t vend = vec ? beg + ((end - beg) & ~(int64_t)3) : beg;
  for (int64_t i = beg + 4 * threadIdx.x; i < vend; i += 4 * OPT_THREADS) {
    const float4 g = *reinterpret_cast<const float4*>(t.grad + i);
    float4 p = *reinterpret_cast<const float4*>(t.param + i);
    float4 m = *reinterpret_cast<const float4*>(t.exp_avg + i);
    float4 v = *reinterpret_cast<const float4*>(t.exp_avg_sq + i);
    upd(g.x, p.x, m.x, v.x); upd(g.y, p.y, m.y, v.y); upd(g.z, p.z, m.z, v.z); upd(g.w, p.w, m.w, v.w);
    *reinterpret_cast<float4*>(t.param + i) = p;
    *reinterpret_cast<float4*>(t.exp_avg + i) = m;
    *reinterpret_cast<float4*>(t.exp_avg_sq + i) = v;
    if (p16) {
      const opt_f32x4_t pv = {p.x, p.y, p.z, p.w};
      *reinterpret_cast<opt_bf16x4_t*>(p16 + i) = __builtin_convertvector(pv, opt_bf16x4_t);
    }
  }
  for (int64_t i = vend + threadIdx.x; i < end; i += OPT_THREADS) {
    upd(t.grad[i], t.param[i], t.exp_avg[i], t.exp_avg_sq[i]);
    if (p16) p16[i] = (__bf16)t.param[i];
  }
}

__device__ __forceinline__ float clip_coef(const float* sumsq, float max_norm) {
  if (!(max_norm > 0.f) || !sumsq) return 1.f;
  const float coef = max_norm / (sqrtf(sumsq[0]) + 1e-6f);
  return coef < 1.f ? coef : 1.f;
}

__global__ __launch_bounds__(OPT_THREADS) void adamw_kernel(const mdemi_tensor_ref* __restrict__ tl,
                                                            const int* __restrict__ chunk_tensor,
                                                            const int* __restrict__ chunk_index, AdamGroups groups,
                                                            const float* __restrict__ sumsq, float max_norm, float gs,
                                                            int step, const int* __restrict__ tensor_steps,
                                                            void* const* __restrict__ p16tab) {
  const int item = blockIdx.x;
  const int ti = chunk_tensor[item];
  const mdemi_tensor_ref t = tl[ti];
  const int64_t beg = (int64_t)chunk_index[item] * OPT_CHUNK;
  const int s = tensor_steps ? tensor_steps[t.step_slot] + 1 : step;
  adamw_item(t, groups.g[t.group], clip_coef(sumsq, max_norm), gs, (float)s, beg, min(t.numel, beg + OPT_CHUNK),
             p16tab ? (__bf16*)p16tab[ti] : nullptr);
}

// capturable form: hyperparameters of step s (= *step_dev, steps already taken)
// from row min(s, nsteps - 1) of a device schedule table
__global__ __launch_bounds__(OPT_THREADS) void adamw_dev_kernel(const mdemi_tensor_ref* __restrict__ tl,
                                                                const int* __restrict__ chunk_tensor,
                                                                const int* __restrict__ chunk_index,
                                                                const mdemi_adamw_group* __restrict__ sched,
                                                                int nsteps, int ngroups,
                                                                const int* __restrict__ step_dev,
                                                                const int* __restrict__ tensor_steps,
                                                                const float* __restrict__ sumsq, float max_norm,
                                                                float gs, void* const* __restrict__ p16tab) {
  const int item = blockIdx.x;
  const int ti = chunk_tensor[item];
  const mdemi_tensor_ref t = tl[ti];
  const int s = step_dev[0];
  const mdemi_adamw_group gp = sched[(int64_t)min(s, nsteps - 1) * ngroups + t.group];
  const int64_t beg = (int64_t)chunk_index[item] * OPT_CHUNK;
  const int bc = tensor_steps ? tensor_steps[t.step_slot] + 1 : s + 1;
  adamw_item(t, gp, clip_coef(sumsq, max_norm), gs, (float)bc, beg, min(t.numel, beg + OPT_CHUNK),
             p16tab ? (__bf16*)p16tab[ti] : nullptr);
}

// after the update: advance the optimizer's step counter and/or every listed
// parameter's own counter (torch's state[p]["step"] += 1 for params with a grad)
__global__ __launch_bounds__(256) void step_tick_kernel(int* step_dev, const mdemi_tensor_ref* __restrict__ tl, int nt,
                                                        int* tensor_steps) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (step_dev && i == 0) step_dev[0] += 1;
  if (tensor_steps && i < nt) tensor_steps[tl[i].step_slot] += 1;
}

}  // namespace mdemi

using namespace mdemi;

extern "C" int mdemi_elementwise(int32_t op, const float* a, const float* b, float* y, int64_t n, float s, float t,
                                 void* stream) {
  MDEMI_REQUIRE(a && y && n >= 0, "elementwise: bad args");
  MDEMI_REQUIRE(op >= 0 && op <= MDEMI_EW_ACT_BWD, "elementwise: bad op %d", op);
  if (op == MDEMI_EW_ADD || op == MDEMI_EW_SIGMOID_SCALE_BWD || op == MDEMI_EW_AXPBY || op == MDEMI_EW_ACT_BWD)
    MDEMI_REQUIRE(b, "elementwise: op %d needs b", op);
  if (n == 0) return MDEMI_OK;
  int64_t nb = cdiv(n, 256);
  nb = nb < 8192 ? nb : 8192;
  hipLaunchKernelGGL(ew_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, op, a, b, y, n, s, t);
  return check_launch("elementwise");
}

namespace mdemi {
typedef __bf16 cast_bf16x8_t __attribute__((ext_vector_type(8)));
typedef float cast_f32x8_t __attribute__((ext_vector_type(8)));
// y = RNE bf16 of x: 8 elements per thread (two 16-B loads, one 16-B store), grid-stride;
// the tail (n % 8) by the first threads one element each
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ x, __bf16* __restrict__ y,
                                                        int64_t n) {
  const int64_t n8 = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(x)[2 * i], b = reinterpret_cast<const float4*>(x)[2 * i + 1];
    const cast_f32x8_t v = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    reinterpret_cast<cast_bf16x8_t*>(y)[i] = __builtin_convertvector(v, cast_bf16x8_t);
  }
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n - 8 * n8) y[8 * n8 + t] = (__bf16)x[8 * n8 + t];
}

// y = a + b and its RNE bf16 copy y16, 4 elements per thread (n % 4 == 0, 16-B aligned)
__global__ __launch_bounds__(256) void add16_kernel(const float4* __restrict__ a, const float4* __restrict__ b,
                                                    float4* __restrict__ y, __bf16* __restrict__ y16, int64_t n4) {
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 u = a[i], v = b[i];
    const float4 o = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
    y[i] = o;
    const f4v ov = {o.x, o.y, o.z, o.w};
    reinterpret_cast<b4*>(y16)[i] = __builtin_convertvector(ov, b4);
  }
}
}  // namespace mdemi

extern "C" int mdemi_add16(const float* a, const float* b, float* y, void* y16, int64_t n, void* stream) {
  MDEMI_REQUIRE(a && b && y && y16 && n >= 0 && n % 4 == 0, "add16: bad args (n %% 4 == 0)");
  MDEMI_REQUIRE(((uintptr_t)a & 15) == 0 && ((uintptr_t)b & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
                    ((uintptr_t)y16 & 7) == 0, "add16: misaligned operand");
  if (n == 0) return MDEMI_OK;
  int64_t nb = cdiv(n / 4, 256);
  nb = nb < 16384 ? nb : 16384;
  hipLaunchKernelGGL(add16_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, (const float4*)a,
                     (const float4*)b, (float4*)y, (__bf16*)y16, n / 4);
  return check_launch("add16");
}

extern "C" int mdemi_cast_bf16(const float* x, void* y, int64_t n, void* stream) {
  MDEMI_REQUIRE(x && y && n >= 0, "cast_bf16: bad args");
  MDEMI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0, "cast_bf16: x and y must be 16-B aligned");
  if (n == 0) return MDEMI_OK;
  int64_t nb = cdiv(std::max<int64_t>(n / 8, 8), 256);
  nb = nb < 16384 ? nb : 16384;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, x, (__bf16*)y, n);
  return check_launch("cast_bf16");
}

namespace mdemi {
size_t colsum_ws_bytes(int64_t rows, int64_t cols) {
  return rows <= COLSUM_ONEPASS ? 0 : align_up((size_t)colsum_blocks_y(rows) * cols * sizeof(float), 256);
}
int colsum_launch_split(const float* x, int64_t rows, int64_t cols, int64_t ld, float* out, float* out2,
                        int64_t split_col, int accumulate, void* ws, hipStream_t st) {
  if (rows <= COLSUM_ONEPASS) {
    hipLaunchKernelGGL(colsum_onepass, dim3((unsigned)cdiv(cols, 32)), dim3(1024), 0, st, x, rows, cols, ld, out,
                       out2, split_col, accumulate);
    return check_launch("colsum");
  }
  const int ny = colsum_blocks_y(rows);
  const int64_t rpb = cdiv(rows, ny);
  dim3 grid((unsigned)cdiv(cols, 32), (unsigned)ny);
  hipLaunchKernelGGL(colsum_partial, grid, dim3(256), 0, st, x, rows, cols, ld, (float*)ws, rpb);
  hipLaunchKernelGGL(colsum_final, dim3((unsigned)cdiv(cols, 256)), dim3(256), 0, st, (const float*)ws, ny, cols, out,
                     out2, split_col, accumulate);
  return check_launch("colsum");
}
int colsum_launch(const float* x, int64_t rows, int64_t cols, int64_t ld, float* out, int accumulate, void* ws,
                  hipStream_t st) {
  return colsum_launch_split(x, rows, cols, ld, out, nullptr, cols, accumulate, ws, st);
}
}  // namespace mdemi

extern "C" size_t mdemi_colsum_workspace_size(int64_t rows, int64_t cols) { return colsum_ws_bytes(rows, cols); }

extern "C" int mdemi_colsum_f32(const float* x, int64_t rows, int64_t cols, int64_t ld, float* out, int accumulate,
                                void* workspace, void* stream) {
  MDEMI_REQUIRE(x && out && rows > 0 && cols > 0 && ld >= cols, "colsum: bad args");
  if (!workspace && colsum_ws_bytes(rows, cols) > 0) { set_error("colsum: workspace required"); return MDEMI_EWORKSPACE; }
  return colsum_launch(x, rows, cols, ld, out, accumulate, workspace, (hipStream_t)stream);
}

// Workspace layout for the optimizer entry points (host computes chunk maps):
//   int chunk_tensor[nitems], int chunk_index[nitems], float part[nitems]
extern "C" size_t mdemi_grad_norm_workspace_size(int32_t nitems) {
  return (size_t)nitems * (2 * sizeof(int) + sizeof(float));
}

extern "C" int mdemi_multi_tensor_chunk(void) { return OPT_CHUNK; }

extern "C" int mdemi_grad_sumsq(const mdemi_tensor_ref* tensors_dev, int32_t ntensors, int64_t nitems,
                                float grad_scale, float* sumsq, void* workspace, void* stream) {
  MDEMI_REQUIRE(tensors_dev && ntensors > 0 && nitems > 0 && sumsq && workspace && grad_scale > 0.f,
                "grad_sumsq: bad args");
  const int* ct = (const int*)workspace;
  const int* ci = ct + nitems;
  float* part = (float*)(ci + nitems);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_partial, dim3((unsigned)nitems), dim3(OPT_THREADS), 0, st, tensors_dev, ntensors, ct, ci,
                     part, grad_scale);
  hipLaunchKernelGGL(sumsq_final, dim3(1), dim3(256), 0, st, part, (int)nitems, sumsq);
  return check_launch("grad_sumsq");
}

extern "C" int mdemi_adamw_step(const mdemi_tensor_ref* tensors_dev, int32_t ntensors,
                                const mdemi_adamw_group* groups_host, int32_t ngroups, const float* sumsq,
                                float max_norm, float grad_scale, int32_t step, int32_t* tensor_steps, int64_t nitems,
                                void* workspace, void* stream) {
  return mdemi_adamw_step16(tensors_dev, ntensors, groups_host, ngroups, sumsq, max_norm, grad_scale, step,
                            tensor_steps, nitems, nullptr, workspace, stream);
}

extern "C" int mdemi_adamw_step16(const mdemi_tensor_ref* tensors_dev, int32_t ntensors,
                                  const mdemi_adamw_group* groups_host, int32_t ngroups, const float* sumsq,
                                  float max_norm, float grad_scale, int32_t step, int32_t* tensor_steps,
                                  int64_t nitems, void* const* param16_dev, void* workspace, void* stream) {
  MDEMI_REQUIRE(tensors_dev && ntensors > 0 && groups_host && ngroups > 0 && ngroups <= 4 &&
                    (step >= 1 || tensor_steps) && nitems > 0 && workspace && grad_scale > 0.f,
                "adamw_step: bad args");
  AdamGroups g;
  for (int i = 0; i < ngroups; ++i) g.g[i] = groups_host[i];
  for (int i = ngroups; i < 4; ++i) g.g[i] = groups_host[0];
  const int* ct = (const int*)workspace;
  const int* ci = ct + nitems;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)nitems), dim3(OPT_THREADS), 0, st, tensors_dev, ct, ci, g, sumsq,
                     max_norm, grad_scale, step, (const int*)tensor_steps, param16_dev);
  if (tensor_steps)
    hipLaunchKernelGGL(step_tick_kernel, dim3((unsigned)cdiv(ntensors, 256)), dim3(256), 0, st, (int*)nullptr,
                       tensors_dev, ntensors, (int*)tensor_steps);
  return check_launch("adamw_step");
}

extern "C" int mdemi_adamw_step_dev(const mdemi_tensor_ref* tensors_dev, int32_t ntensors,
                                    const mdemi_adamw_group* sched_dev, int32_t nsteps, int32_t ngroups,
                                    int32_t* step_dev, int32_t* tensor_steps, const float* sumsq, float max_norm,
                                    float grad_scale, int64_t nitems, void* workspace, void* stream) {
  return mdemi_adamw_step_dev16(tensors_dev, ntensors, sched_dev, nsteps, ngroups, step_dev, tensor_steps, sumsq,
                                max_norm, grad_scale, nitems, nullptr, workspace, stream);
}

extern "C" int mdemi_adamw_step_dev16(const mdemi_tensor_ref* tensors_dev, int32_t ntensors,
                                      const mdemi_adamw_group* sched_dev, int32_t nsteps, int32_t ngroups,
                                      int32_t* step_dev, int32_t* tensor_steps, const float* sumsq, float max_norm,
                                      float grad_scale, int64_t nitems, void* const* param16_dev, void* workspace,
                                      void* stream) {
  MDEMI_REQUIRE(tensors_dev && ntensors > 0 && sched_dev && nsteps > 0 && ngroups > 0 && ngroups <= 4 && step_dev &&
                    nitems > 0 && workspace && grad_scale > 0.f,
                "adamw_step_dev: bad args");
  const int* ct = (const int*)workspace;
  const int* ci = ct + nitems;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adamw_dev_kernel, dim3((unsigned)nitems), dim3(OPT_THREADS), 0, st, tensors_dev, ct, ci, sched_dev,
                     nsteps, ngroups, (const int*)step_dev, (const int*)tensor_steps, sumsq, max_norm, grad_scale,
                     param16_dev);
  hipLaunchKernelGGL(step_tick_kernel, dim3((unsigned)cdiv(ntensors, 256)), dim3(256), 0, st, (int*)step_dev,
                     tensors_dev, ntensors, (int*)tensor_steps);
  return check_launch("adamw_step_dev");
}

// Stochastic depth (timm DropPath, swin_transformer.py:181,243-244):
// y = (a ? a : 0) + b * scale[row / rows_per_group]  (scale = keep/(1-p) per sample)
namespace mdemi {
__global__ __launch_bounds__(256) void rowscale_add_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                           const float* __restrict__ scale, float* __restrict__ y,
                                                           int64_t per_group, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float s = scale[i / per_group];
    y[i] = (a ? a[i] : 0.f) + b[i] * s;
  }
}
}  // namespace mdemi

extern "C" int mdemi_rowscale_add(const float* a, const float* b, const float* scale, float* y, int64_t per_group,
                                  int64_t n, void* stream) {
  MDEMI_REQUIRE(b && scale && y && per_group > 0 && n >= 0, "rowscale_add: bad args");
  if (n == 0) return MDEMI_OK;
  int64_t nb = cdiv(n, 256);
  nb = nb < 8192 ? nb : 8192;
  hipLaunchKernelGGL(rowscale_add_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, a, b, scale, y,
                     per_group, n);
  return check_launch("rowscale_add");
}
