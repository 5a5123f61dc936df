/*
 * mdemi.h — C ABI of libmdemi.so, the MI355X (gfx950) kernel library behind the
 * dense-depth train/inference hot path of pitlover/Monocular-Depth-Estimation.
 *
 * The reference has no native code or FFI: every op on its hot path is an ATen
 * op called from the model modules.  Each entry point below replaces the ATen
 * op(s) that one reference call site runs; the replaced call site is cited
 * (paths relative to the reference root).  The Python mirror of the
 * reference's module surface (monocular-depth-estimation_amd/mdemi) binds these
 * with ctypes; INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *  - All tensors are fp32, dense, device pointers owned by the caller
 *    (PyTorch's caching allocator).  The library never allocates or frees
 *    device memory; entries that need scratch take a workspace pointer whose
 *    size comes from the matching *_workspace_size() query.
 *  - `stream` is a hipStream_t passed as void*; every call is stream-ordered,
 *    asynchronous, reentrant and never synchronises the device.
 *  - Return value: 0 on success, a negative MDEMI_E* code otherwise.
 *    mdemi_last_error() returns a thread-local message for the last failure.
 *  - Activations inside the library are channels-last (NHWC / token-major
 *    [rows, C]); the reference's NCHW tensors are converted at the model
 *    boundary only.
 */
#ifndef MDEMI_H
#define MDEMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDEMI_OK 0
#define MDEMI_EINVAL (-1)   /* bad argument / shape */
#define MDEMI_ELAUNCH (-2)  /* HIP launch failure */
#define MDEMI_EUNSUP (-3)   /* unsupported configuration */
#define MDEMI_EWORKSPACE (-4) /* workspace missing or too small */

const char* mdemi_last_error(void);
int mdemi_version(void);

/* ------------------------------------------------------------------------ */
/* GEMM family (fp32 in / fp32 accumulate on v_mfma_f32_32x32x2_f32).        */
/* Replaces nn.Linear (addmm) in swin_transformer.py:18-20,104,106,259,      */
/* newcrf_layers.py:16-20,102,104, luna_layer.py:149-158, miniViT.py:19-23,  */
/* and — through the implicit-im2col operand layout — nn.Conv2d in          */
/* newcrf_layers.py:384,389, uper_crf_head.py:38-44,341-348,                  */
/* NewCRFDepth.py:155, unet_adaptive_bins.py:12-17,32,42,88-91,              */
/* miniViT.py:17-18, layers.py:15-20, layer_utils.py:20-24.                  */
/*                                                                          */
/*   C[b][i][j] = act( alpha * sum_k A(b,i,k) * B(b,k,j) + bias + beta*C )   */
/*                (+ residual[b][i][j])                                       */
/* ------------------------------------------------------------------------ */

/* operand layouts */
#define MDEMI_L_KCONTIG 0  /* A stored [i][k] (lda = row stride);  B stored [j][k] */
#define MDEMI_L_MNCONTIG 1 /* A stored [k][i];                      B stored [k][j] */
#define MDEMI_L_CONV 2     /* implicit im2col of an NHWC activation (see conv geom):
                              A: i = output pixel, k = (ky,kx,c)
                              B: k = output pixel, j = (ky,kx,c)                */
/* operand element transforms applied while loading */
#define MDEMI_OP_NONE 0
#define MDEMI_OP_GELU 1    /* exact erf GELU (nn.GELU default) */
/* bias modes */
#define MDEMI_BIAS_NONE 0
#define MDEMI_BIAS_COL 1   /* bias[j] */
#define MDEMI_BIAS_ROW 2   /* bias[i] */
/* epilogue activations */
#define MDEMI_ACT_NONE 0
#define MDEMI_ACT_GELU 1
#define MDEMI_ACT_RELU 2
#define MDEMI_ACT_LEAKY 3      /* negative slope 0.01 (nn.LeakyReLU default) */
#define MDEMI_ACT_GELU_GRAD 4  /* out = acc * gelu'(aux[i][j])                 */
#define MDEMI_ACT_SIGMOID 5
#define MDEMI_ACT_SILU 6       /* x * sigmoid(x) (nn.SiLU: decoder_v8.py:24; EfficientNet swish) */
#define MDEMI_ACT_RELU_GRAD 7  /* out = acc * [aux[i][j] > 0]                  */
#define MDEMI_ACT_SILU_GRAD 8  /* out = acc * silu'(aux[i][j])                 */
/* conv padding modes */
#define MDEMI_PAD_ZERO 0
#define MDEMI_PAD_REPLICATE 1

typedef struct mdemi_conv_geom {
  int32_t n, h, w, c;       /* input activation, NHWC */
  int32_t oh, ow;           /* output spatial size */
  int32_t kh, kw, stride, pad;  /* pad = top/left padding; may be negative (a crop,
                                  the dgrad of a padded 1x1 conv, unet_adaptive_bins.py:32);
                                  bottom/right padding follows from oh/ow (TF 'same') */
  int32_t pad_mode;         /* MDEMI_PAD_* */
  int32_t _reserved;
} mdemi_conv_geom;

typedef struct mdemi_gemm_desc {
  int32_t M, N, K, batch;
  const float* A; int64_t lda; int64_t a_bstride; int32_t a_layout; int32_t a_op;
  const float* B; int64_t ldb; int64_t b_bstride; int32_t b_layout; int32_t b_op;
  float* C; int64_t ldc; int64_t c_bstride;
  float alpha, beta;
  const float* bias; int32_t bias_mode; int32_t act;
  const float* aux; int64_t ldaux; int64_t aux_bstride;       /* MDEMI_ACT_GELU_GRAD */
  const float* residual; int64_t ldres; int64_t res_bstride;  /* added after act */
  int32_t split_k; int32_t _pad0;  /* >1: K split over workgroups, fp32 slabs in workspace */
  void* workspace; int64_t workspace_bytes;
  mdemi_conv_geom conv;            /* geometry for an MDEMI_L_CONV operand */
  float* preact; int64_t ldpre; int64_t pre_bstride;  /* optional 2nd output: the value
                                      before `act` (and before residual); lets fc1 store
                                      both h and gelu(h) in one pass */
  float* rowsum_a;                 /* optional [M] output: sum_k A(i,k), A m-contiguous and
                                      batch 1 -- the bias gradient of a weight-gradient GEMM
                                      (dW = dY^T X, db = dY^T 1) without a second pass over dY */
  int32_t batch_inner; int32_t _pad1;  /* > 1: batch index z = o * batch_inner + i, operand
                                      offsets o * X_bstride + i * X_bstride_inner -- one
                                      launch for every (image, head) of a multi-head
                                      attention GEMM (heads are column slices of the token
                                      buffers).  0/1: one-level batch.  Needs batch %
                                      batch_inner == 0 and no aux/residual/preact/rowsum_a */
  int64_t a_bstride_inner, b_bstride_inner, c_bstride_inner;
  const float* row_scale; int64_t row_scale_group;  /* optional: the value after `act`
                                      is multiplied by row_scale[i / row_scale_group]
                                      before the residual add -- timm DropPath's per-sample
                                      keep/(1-p) scale of a residual branch
                                      (swin_transformer.py:232,239) fused into the proj /
                                      fc2 epilogue.  Batch 1. */
} mdemi_gemm_desc;

size_t mdemi_gemm_workspace_size(const mdemi_gemm_desc* d);
int mdemi_gemm_f32(const mdemi_gemm_desc* d, void* stream);
/* Same contract with bf16 compute (mixed precision, BASELINE configs[4] "bf16"
 * = torch.autocast's matmul numerics): fp32 operands are rounded to bf16 (RNE)
 * as they are staged, products run on the bf16 MFMA with fp32 accumulation,
 * and the fp32 epilogue and output are those of mdemi_gemm_f32.  Replaces the
 * autocast bf16 addmm/bmm/conv of the reference's layers (e.g.
 * model/Depthformer/luna_layer.py:181-259, layer_utils.py:6-34) for the
 * mixed-precision train step.  Workspace: mdemi_gemm_workspace_size. */
int mdemi_gemm_bf16(const mdemi_gemm_desc* d, void* stream);
/* Same contract at fp32 accuracy on the bf16 matrix cores ("f32e"): each fp32
 * operand is split exactly into three bf16 planes (a = a_hi + a_mid + a_lo, RNE)
 * as it is staged and the six products hi.hi, hi.mid, mid.hi, hi.lo, lo.hi,
 * mid.mid run on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (dropped terms
 * below 2^-24 |a||b|), at 2.67x the fp32 matrix-core peak.  fp32-level error
 * except on heavily cancelling sums, where the bf16 MFMA's accumulation is
 * measurably less exact than mdemi_gemm_f32's: an opt-in.  Replaces the same fp32 nn.Linear / nn.Conv2d / bmm products
 * as mdemi_gemm_f32 (swin_transformer.py:18-20,104,106,259; newcrf_layers.py:
 * 16-20,102,104,384,389; uper_crf_head.py:38-44,341-348; ...). */
int mdemi_gemm_f32e(const mdemi_gemm_desc* d, void* stream);
/* bf16 storage path of precision "bf16" (BASELINE configs[4]): the same contract as
 * mdemi_gemm_bf16 with the operands given as bf16 tensors (a16, b16: 16-bit RNE copies of
 * A and B, same layouts, leading dimensions and strides in elements) DMA'd straight into
 * LDS, so an activation or weight stored in bf16 is read at 2 B per element with no
 * conversion; results are bit-identical to mdemi_gemm_bf16 on the fp32 tensors whose RNE
 * bf16 a16/b16 are.  c16 (optional, may be NULL): a bf16 (RNE) copy of the final output,
 * C's layout, written by the same epilogue (the bf16 operand of a later GEMM).  Layouts
 * the bf16 loaders cannot stage (K / extent / C not a multiple of 8, a load-time op,
 * rowsum_a) fall back to mdemi_gemm_bf16 on d->A / d->B, which must then be given.
 * Replaces the autocast bf16 conv/linear/bmm of model/Depthformer/layer_utils.py:6-34,
 * luna_layer.py:181-259, decoder_v8.py:97-171. */
int mdemi_gemm_bf16x(const mdemi_gemm_desc* d, const void* a16, const void* b16, void* c16, void* stream);
/* y[i] = RNE bf16 of x[i] (n elements; x, y 16-B aligned): the bf16 copy of an fp32 operand
 * that no producer wrote in bf16 (precision "bf16" GEMM operands, mdemi_gemm_bf16x). */
int mdemi_cast_bf16(const float* x, void* y, int64_t n, void* stream);
/* y = a + b with its RNE bf16 copy y16 (n % 4 == 0): a residual sum that the next bf16 GEMM
 * reads as its operand (the bf16 storage path). */
int mdemi_add16(const float* a, const float* b, float* y, void* y16, int64_t n, void* stream);
/* 1 when mdemi_gemm_bf16x would take the bf16-operand path for this descriptor. */
int mdemi_gemm_bf16x_supported(const mdemi_gemm_desc* d, const void* a16, const void* b16);
/* tuning hook of the bf16-operand family: 0 = 128-row tile, 1 = 256-row tile, 2 = 128-row tile
 * with two K tiles per LDS stage, -1 = per-shape autotune (default; all bit-identical). */
int mdemi_gemm_set_variant_b16(int32_t variant);
/* tuning hook: pipelining variant (0..5, see gemm_f32.hip; -1 = time the
 * candidates once per distinct shape and cache the winner, the default -- all
 * variants produce bit-identical results) and tile raster (group_m > 0:
 * XCD-aware grouped raster, 0: plain).  Process-global. */
int mdemi_gemm_set_variant(int32_t variant, int32_t group_m);
/* tuning hook of the 16-bit family (mdemi_gemm_bf16 / mdemi_gemm_f32e): 0 = 128-row
 * tile with two LDS buffers, 1 = one buffer, 2 = 256-row tile; -1 = per-shape
 * autotune (default; all bit-identical). */
int mdemi_gemm_set_variant_m16(int32_t variant);
/* scheduling switches of the fp32 family (process-global; defaults from the environment:
 * MDEMI_GEMM_TAIL_SPLIT, on unless 0; MDEMI_GEMM_INLINE_REDUCE, off unless 1): tail_split --
 * a whole-K GEMM whose tiles leave a thin last round of workgroups splits the rows of the
 * leftover tiles over K (a plan that depends on the shape only); inline_reduce -- split-K
 * slabs are combined by the last-arriving piece of each tile instead of a separate reduce
 * launch (bit-identical either way; the bf16 families follow MDEMI_GEMM_INLINE_REDUCE_B16). */
int mdemi_gemm_set_options(int32_t tail_split, int32_t inline_reduce);

/* column / row sums (bias gradients: db[j] = sum_i dY[i][j])
 * replaces the bias-grad reduction autograd runs for every nn.Linear/Conv2d. */
size_t mdemi_colsum_workspace_size(int64_t rows, int64_t cols);
int mdemi_colsum_f32(const float* x, int64_t rows, int64_t cols, int64_t ld,
                     float* out, int accumulate, void* workspace, void* stream);

/* KxK 'same' conv to ONE output channel over NHWC (DispHead.conv1,
 * NewCRFDepth.py:155): memory-bound sweep instead of an N=1 GEMM.  w is in the
 * reference layout [1][C][K][K]; dx/dw/db may be NULL to skip that gradient. */
int mdemi_headconv_fwd(const float* x, const float* w, const float* b, float* y, int32_t N,
                       int32_t H, int32_t W, int32_t C, int32_t K, int32_t pad, void* stream);
size_t mdemi_headconv_wgrad_workspace_size(int32_t N, int32_t H, int32_t W, int32_t C, int32_t K);
int mdemi_headconv_bwd(const float* dy, const float* x, const float* w, float* dx, float* dw,
                       float* db, int32_t N, int32_t H, int32_t W, int32_t C, int32_t K, int32_t pad,
                       void* workspace, void* stream);

/* ------------------------------------------------------------------------ */
/* Adaptive-bin depth head (unet_adaptive_bins.py:97-107,                   */
/* depthformer_v8.py:62-73, decoder_v8.py:158-159):                          */
/*   p = softmax_k(logits[b,k,:]),  pred[b,:] = sum_k p_k * centers[b,k]     */
/* logits NCHW-contiguous [B][K][HW]; stats [B][2][HW] = (max, 1/sum) saved  */
/* for the backward.  do_softmax=0 means `logits` already hold probabilities */
/* (Depthformer v8 applies the softmax inside the decoder, decoder_v8.py:159) */
/* ------------------------------------------------------------------------ */
int mdemi_binhead_fwd(const float* logits, const float* centers, float* pred,
                      float* stats, float* probs_out, int32_t B, int32_t K, int64_t HW,
                      int32_t do_softmax, void* stream);
size_t mdemi_binhead_bwd_workspace_size(int32_t B, int32_t K, int64_t HW);
int mdemi_binhead_bwd(const float* logits, const float* centers, const float* pred,
                      const float* stats, const float* dpred, float* dlogits,
                      float* dcenters, int32_t B, int32_t K, int64_t HW, int32_t do_softmax,
                      void* workspace, void* stream);

/* ------------------------------------------------------------------------ */
/* LayerNorm over the last dim (nn.LayerNorm, eps configurable):             */
/* swin_transformer.py:176,182,260,416,541; newcrf_layers.py:182,188,413;    */
/* luna_layer.py:153-155; feed_forward.py:21.                                */
/* ------------------------------------------------------------------------ */
int mdemi_layernorm_fwd(const float* x, const float* gamma, const float* beta,
                        float* y, float* mean, float* rstd, int64_t rows, int32_t C,
                        float eps, void* stream);
/* The same, also writing y16 (optional, 8-B aligned): the RNE bf16 copy of y that a bf16
 * GEMM reading the normalised rows takes as its operand (bf16 storage; luna_layer.py:202-250
 * and feed_forward.py:29-46 under torch.autocast, configs[4]). */
int mdemi_layernorm_fwd16(const float* x, const float* gamma, const float* beta, float* y, void* y16,
                          float* mean, float* rstd, int64_t rows, int32_t C, float eps, void* stream);
size_t mdemi_layernorm_bwd_workspace_size(int64_t rows, int32_t C);
int mdemi_layernorm_bwd(const float* dy, const float* x, const float* mean,
                        const float* rstd, const float* gamma, float* dx,
                        float* dgamma, float* dbeta, int64_t rows, int32_t C,
                        int32_t accumulate_dx, void* workspace, void* stream);
/* Backward of a LayerNorm whose input also feeds a residual (skip) path,
 * x -> (LN(x), x) in swin_transformer.py:200-245 / newcrf_layers.py:204-257:
 * dx = LN'(dy) + dadd with dadd the skip path's gradient (may alias dx), so
 * the two gradient contributions are summed in the same sweep. */
int mdemi_layernorm_bwd_add(const float* dy, const float* x, const float* mean,
                            const float* rstd, const float* gamma, const float* dadd, float* dx,
                            float* dgamma, float* dbeta, int64_t rows, int32_t C,
                            void* workspace, void* stream);

/* ------------------------------------------------------------------------ */
/* (Shifted-)window multi-head attention with relative position bias.       */
/* Folds F.pad / torch.roll / window_partition / window_reverse / crop of   */
/* swin_transformer.py:201-240 and newcrf_layers.py:207-251 into the load/  */
/* store index maps, the SW-MSA mask of swin_transformer.py:361-380 into an  */
/* in-kernel region test, and computes WindowAttention.forward               */
/* (swin_transformer.py:112-144 minus the qkv/proj Linears;                  */
/*  newcrf_layers.py:110-149 minus qk/proj).                                  */
/* q,k,v,out, dq,dk,dv are token-major rows of the UNPADDED [B,H,W] grid.    */
/* Pad tokens take the value of *_pad (the Linear's bias, because the        */
/* reference pads after norm1 so pad rows of qkv(0) == bias) or 0 if NULL.   */
/* ------------------------------------------------------------------------ */
typedef struct mdemi_winattn_desc {
  int32_t B, H, W, heads, head_dim, window, shift, _pad0;
  float scale;
  int32_t _pad1;
  const float* q; const float* k; int64_t qk_ld;
  const float* q_pad; const float* k_pad;
  const float* v; int64_t v_ld; const float* v_pad;
  const float* rpb_table;          /* [(2w-1)^2][heads] */
  float* out; int64_t out_ld;     /* forward output; the backward reads it (D = rowsum(dO*O)) */
  float* lse;                      /* [nwin][heads][window^2] row log-sum-exp: written by the
                                      forward (may be NULL there), required by the backward */
  /* backward only */
  const float* dout;
  float* dq; float* dk; int64_t dqk_ld;
  float* dv; int64_t dv_ld;
  float* d_rpb_table;              /* [(2w-1)^2][heads], overwritten */
  float* dq_pad; float* dk_pad; float* dv_pad;   /* [C] sums over pad tokens, overwritten (may be NULL) */
  void* workspace; int64_t workspace_bytes;
} mdemi_winattn_desc;

size_t mdemi_winattn_fwd_workspace_size(const mdemi_winattn_desc* d);
int mdemi_winattn_fwd(const mdemi_winattn_desc* d, void* stream);
size_t mdemi_winattn_bwd_workspace_size(const mdemi_winattn_desc* d);
int mdemi_winattn_bwd(const mdemi_winattn_desc* d, void* stream);
/* The same backward reusing the forward's expanded relative-position bias: bias_expanded =
 * the first mdemi_winattn_fwd_workspace_size() bytes of the forward call's workspace, kept
 * unchanged since (the table it expands is the same parameter); null = expand it again.
 * One launch fewer per backward (WindowAttention.forward, swin_transformer.py:112-144). */
int mdemi_winattn_bwd_bias(const mdemi_winattn_desc* d, const float* bias_expanded, void* stream);

/* ------------------------------------------------------------------------ */
/* Scale-invariant log loss (restated; the reference's loss module is        */
/* missing — config keys loss.alpha/beta/per_image, e.g.                     */
/* json/nyu/newcrfs/newcrfs_github_eval.json).                               */
/*   g = log(pred) - log(gt) on gt > min_depth                               */
/*   L_group = alpha * sqrt(Var(g) + beta * mean(g)^2)                       */
/* groups = images (per_image) or the whole batch; loss = mean over groups.  */
/* loss[0] receives the scalar; stats keeps (n, sum g, sum g^2) per group.   */
/* ------------------------------------------------------------------------ */
size_t mdemi_silog_workspace_size(int32_t B, int64_t HW);
int mdemi_silog_fwd(const float* pred, const float* gt, float* loss, float* stats,
                    int32_t B, int64_t HW, float min_depth, float alpha, float beta,
                    int32_t per_image, int32_t unbiased, void* workspace, void* stream);
int mdemi_silog_bwd(const float* pred, const float* gt, const float* stats,
                    const float* dloss, float* dpred, int32_t B, int64_t HW,
                    float min_depth, float alpha, float beta, int32_t per_image,
                    int32_t unbiased, void* stream);

/* ------------------------------------------------------------------------ */
/* Resampling / layout sweeps (HBM-bound).                                   */
/* ------------------------------------------------------------------------ */
/* Bilinear resize, NHWC (F.interpolate mode='bilinear': NewCRFDepth.py:185-188,
 * uper_crf_head.py:51-55, unet_adaptive_bins.py:22, layer_utils.py:110-115,
 * decoder_v8.py:149-152).  scale_h/scale_w > 0 override the size-derived
 * ratio (align_corners=False with scale_factor, as F.interpolate computes it).
 * out may be a channel slice of a wider buffer: out_cstride = its row pitch. */
int mdemi_bilinear_fwd(const float* x, float* out, int32_t N, int32_t H, int32_t W,
                       int32_t C, int32_t OH, int32_t OW, int32_t align_corners,
                       float scale_h, float scale_w, int64_t in_cstride,
                       int64_t out_cstride, void* stream);
int mdemi_bilinear_bwd(const float* dout, float* dx, int32_t N, int32_t H, int32_t W,
                       int32_t C, int32_t OH, int32_t OW, int32_t align_corners,
                       float scale_h, float scale_w, int64_t dout_cstride,
                       int64_t dx_cstride, int32_t accumulate, void* stream);

/* Layout conversions (NCHW <-> NHWC), PixelShuffle as an NHWC index map
 * (NewCRFDepth.py:132,134,136), patchify for the stride==kernel PatchEmbed
 * conv (swin_transformer.py:420-436, layers.py:15-20). */
int mdemi_nchw_to_nhwc(const float* x, float* y, int32_t N, int32_t C, int64_t HW, void* stream);
int mdemi_nhwc_to_nchw(const float* x, float* y, int32_t N, int32_t C, int64_t HW, void* stream);
int mdemi_pixel_shuffle_nhwc(const float* x, float* y, int32_t N, int32_t H, int32_t W,
                             int32_t C, int32_t r, int32_t inverse, void* stream);
int mdemi_patchify_nchw(const float* img, float* cols, int32_t N, int32_t C, int32_t H,
                        int32_t W, int32_t p, int32_t inverse, void* stream);

/* PatchMerging 2x2 gather (swin_transformer.py:272-284): [N,H,W,C] ->
 * [N,ceil(H/2),ceil(W/2),4C] in the reference's (0,0),(1,0),(0,1),(1,1) order,
 * zero-padded for odd sizes.  inverse=1 writes the adjoint into x (from y). */
int mdemi_space_to_depth2(const float* x, float* y, int32_t N, int32_t H, int32_t W, int32_t C,
                          int32_t inverse, void* stream);
/* strided 2-D copy (channel-slice concat/split, torch.cat in uper_crf_head.py:355,
 * unet_adaptive_bins.py:23, layer_utils.py:116) */
int mdemi_copy2d(const float* src, int64_t src_ld, float* dst, int64_t dst_ld, int64_t rows,
                 int64_t cols, int32_t accumulate, void* stream);

/* adaptive average pooling, NHWC (nn.AdaptiveAvgPool2d, uper_crf_head.py:38) */
int mdemi_adaptive_avgpool_fwd(const float* x, float* y, int32_t N, int32_t H, int32_t W,
                               int32_t C, int32_t OH, int32_t OW, void* stream);
int mdemi_adaptive_avgpool_bwd(const float* dy, float* dx, int32_t N, int32_t H, int32_t W,
                               int32_t C, int32_t OH, int32_t OW, void* stream);

/* ------------------------------------------------------------------------ */
/* Channel normalisation over NHWC activations (training-mode statistics):  */
/* BatchNorm2d (uper_crf_head.py:341-348 via ConvModule, unet_adaptive_bins  */
/* .py:13,16, layer_utils.py:25) and GroupNorm (uper_crf_head.py:35).        */
/* groups == C for BatchNorm (statistics over N,H,W per channel); for         */
/* GroupNorm statistics are per (n, group) over H,W and C/groups channels.   */
/* act: MDEMI_ACT_NONE / RELU / LEAKY / GELU fused after the affine.          */
/* ------------------------------------------------------------------------ */
size_t mdemi_chnorm_workspace_size(int32_t N, int64_t HW, int32_t C, int32_t groups, int32_t is_bn);
int mdemi_chnorm_fwd(const float* x, const float* gamma, const float* beta, float* y,
                     float* mean, float* rstd, int32_t N, int64_t HW, int32_t C,
                     int32_t groups, int32_t is_bn, float eps, int32_t act,
                     void* workspace, void* stream);
int mdemi_chnorm_bwd(const float* dy, const float* x, const float* y, const float* mean,
                     const float* rstd, const float* gamma, const float* beta, float* dx,
                     float* dgamma, float* dbeta, int32_t N, int64_t HW, int32_t C,
                     int32_t groups, int32_t is_bn, int32_t act, void* workspace, void* stream);

/* inference-mode normalisation with caller-supplied statistics (BN eval) */
int mdemi_chnorm_apply(const float* x, const float* gamma, const float* beta, const float* mean,
                       const float* rstd, float* y, int32_t N, int64_t HW, int32_t C, int32_t groups,
                       int32_t is_bn, int32_t act, void* stream);
/* training-mode BatchNorm2d forward (mdemi_chnorm_fwd with is_bn = 1) that also applies the
 * running-statistics update of mdemi_bn_running_update (momentum, num_batches_tracked += 1
 * when given) inside its statistics pass: nn.BatchNorm2d.forward in train mode in one call
 * (uper_crf_head.py:341-348 ConvModule, unet_adaptive_bins.py:13,16, layer_utils.py:25). */
int mdemi_bn_train_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean,
                       float* rstd, float* running_mean, float* running_var, int64_t* num_batches_tracked,
                       float momentum, int32_t N, int64_t HW, int32_t C, float eps, int32_t act,
                       void* workspace, void* stream);
/* the same, also writing y16 (may be NULL): the RNE bf16 copy of y that a following bf16 GEMM
 * reads (the bf16 storage path of precision "bf16", layer_utils.py:6-34 ConvBN -> conv). */
int mdemi_bn_train_fwd16(const float* x, const float* gamma, const float* beta, float* y, void* y16,
                         float* mean, float* rstd, float* running_mean, float* running_var,
                         int64_t* num_batches_tracked, float momentum, int32_t N, int64_t HW, int32_t C,
                         float eps, int32_t act, void* workspace, void* stream);
/* mdemi_bn_train_fwd16 that also writes pooled [N][C] = the spatial mean of y per image (the
 * SqueezeExcite pooling of the EfficientNet block whose BatchNormAct2d output feeds its SE,
 * gen-efficientnet via unet_adaptive_bins.py:129 / depthformer_v8.py:89) in the same sweep
 * as y.  C % 4 == 0, 16-B aligned x / y; workspace: mdemi_bn_train_fwd_pooled_workspace_size. */
size_t mdemi_bn_train_fwd_pooled_workspace_size(int32_t N, int64_t HW, int32_t C);
int mdemi_bn_train_fwd_pooled(const float* x, const float* gamma, const float* beta, float* y, void* y16,
                              float* pooled, float* mean, float* rstd, float* running_mean, float* running_var,
                              int64_t* num_batches_tracked, float momentum, int32_t N, int64_t HW, int32_t C,
                              float eps, int32_t act, void* workspace, void* stream);
/* mdemi_chnorm_bwd (BatchNorm) also writing dx16 (may be NULL): the RNE bf16 copy of dx, the
 * output gradient of the conv before the BN that its data- and weight-gradient GEMMs read. */
int mdemi_chnorm_bwd16(const float* dy, const float* x, const float* y, const float* mean,
                       const float* rstd, const float* gamma, const float* beta, float* dx, void* dx16,
                       float* dgamma, float* dbeta, int32_t N, int64_t HW, int32_t C,
                       int32_t groups, int32_t is_bn, int32_t act, void* workspace, void* stream);
/* backward of mdemi_chnorm_apply for BatchNorm (eval-mode BN inside a training step:
 * frozen statistics, so dx = gamma * rstd * act'(pre) * dy with no batch terms);
 * dx may be NULL (input needs no gradient); dgamma and dbeta are both NULL (frozen
 * affine) or both set, and then need mdemi_chnorm_workspace_size(..., is_bn=1) bytes.
 * Replaces autograd through F.batch_norm(training=False) where the reference trains
 * with BatchNorm layers in eval mode (unet_adaptive_bins.py freeze, layer_utils.py). */
int mdemi_bn_frozen_bwd(const float* dy, const float* x, const float* mean, const float* rstd,
                        const float* gamma, const float* beta, float* dx, float* dgamma, float* dbeta,
                        int32_t N, int64_t HW, int32_t C, int32_t act, void* workspace, void* stream);
/* BatchNorm2d running-statistics update in training (nn.BatchNorm2d
 * semantics: unbiased batch variance, running = (1-m) running + m batch), from
 * the batch mean / rstd of mdemi_chnorm_fwd over `rows` = N*H*W samples, and
 * num_batches_tracked += 1 when that pointer is given. One launch instead of the
 * per-layer chain of small tensor ops (uper_crf_head.py:341-348,
 * unet_adaptive_bins.py:13,16, layer_utils.py:25). */
int mdemi_bn_running_update(const float* mean, const float* rstd, float* running_mean, float* running_var,
                            int64_t* num_batches_tracked, int32_t C, int64_t rows, float eps, float momentum,
                            void* stream);

/* ------------------------------------------------------------------------ */
/* Elementwise helpers                                                       */
/* ------------------------------------------------------------------------ */
#define MDEMI_EW_ADD 0        /* y = a + b */
#define MDEMI_EW_SIGMOID_SCALE 1  /* y = sigmoid(a) * s */
#define MDEMI_EW_SIGMOID_SCALE_BWD 2 /* y = b * s * sig(a)(1-sig(a)) with a = pre-activation */
#define MDEMI_EW_AXPBY 3      /* y = s*a + t*b */
#define MDEMI_EW_ACT_BWD 4    /* y = b * act'(a), act given in `s` as an MDEMI_ACT_* code */
int mdemi_elementwise(int32_t op, const float* a, const float* b, float* y, int64_t n,
                      float s, float t, void* stream);
/* stochastic depth residual (timm DropPath, swin_transformer.py:243-244):
 * y = (a ? a : 0) + b * scale[i / per_group] */
int mdemi_rowscale_add(const float* a, const float* b, const float* scale, float* y,
                       int64_t per_group, int64_t n, void* stream);

/* ------------------------------------------------------------------------ */
/* Optimizer (restated; reference run.py is missing): multi-tensor AdamW    */
/* with the global-norm gradient clip (clip_grad_norm_, cfg train.grad_norm)  */
/* folded into the update — no host synchronisation.                          */
/* ------------------------------------------------------------------------ */
typedef struct mdemi_tensor_ref {
  float* param; float* grad; float* exp_avg; float* exp_avg_sq;
  int64_t numel; int32_t group;
  int32_t step_slot;  /* index of this parameter's counter in tensor_steps (below) */
} mdemi_tensor_ref;

typedef struct mdemi_adamw_group {
  float lr, beta1, beta2, eps, weight_decay;
  int32_t _pad;
} mdemi_adamw_group;

/* Work is split into (tensor, chunk) items of mdemi_multi_tensor_chunk()
 * elements.  The caller builds the item maps once (int chunk_tensor[nitems],
 * int chunk_index[nitems]) at the start of the workspace; the float partials
 * follow.  tensors_dev is a device array of mdemi_tensor_ref. */
int mdemi_multi_tensor_chunk(void);
size_t mdemi_grad_norm_workspace_size(int32_t nitems);
/* sumsq[0] <- sum over tensors of ||grad_scale * grad||^2 (deterministic two-level sum).
 * grad_scale (> 0) is the factor every gradient is taken at, in this norm and in the
 * update below: 1/world folds the data-parallel mean into the optimizer (the summed
 * gradients of the all-reduce are never swept just to scale them); 1 otherwise. */
int mdemi_grad_sumsq(const mdemi_tensor_ref* tensors_dev, int32_t ntensors, int64_t nitems,
                     float grad_scale, float* sumsq, void* workspace, void* stream);
/* One AdamW step (torch.optim.AdamW semantics, decoupled weight decay).
 * groups_host: up to 4 parameter groups (host memory, passed by value).
 * step: 1-based step count for bias correction.  max_norm <= 0 disables the
 * clip; otherwise grads (times grad_scale) are scaled by min(1, max_norm / (sqrt(sumsq)+1e-6)),
 * as torch.nn.utils.clip_grad_norm_ does, without a host round trip.
 * tensor_steps (device, optional): per-parameter step counters, torch's
 * state[p]["step"] -- a parameter whose gradient first appears late has its own
 * count.  When given, parameter t's bias corrections use
 * tensor_steps[t.step_slot] + 1 (and `step` is ignored), and a trailing kernel
 * increments tensor_steps[t.step_slot] for every tensor in the table. */
int mdemi_adamw_step(const mdemi_tensor_ref* tensors_dev, int32_t ntensors,
                     const mdemi_adamw_group* groups_host, int32_t ngroups,
                     const float* sumsq, float max_norm, float grad_scale, int32_t step,
                     int32_t* tensor_steps, int64_t nitems, void* workspace, void* stream);
/* Capturable form (a hipGraph-captured train step): the hyperparameters come
 * from device memory.  sched_dev is a [nsteps][ngroups] table of
 * mdemi_adamw_group entries -- e.g. the OneCycle lr / beta1 of every optimizer step --
 * *step_dev the number of optimizer steps already taken: the update uses row
 * min(*step_dev, nsteps - 1) and bias corrections for step *step_dev + 1 (or, with
 * tensor_steps, tensor_steps[t.step_slot] + 1 per parameter), then a trailing
 * kernel increments *step_dev (and the per-parameter counters).  Same numerics
 * as mdemi_adamw_step. */
int mdemi_adamw_step_dev(const mdemi_tensor_ref* tensors_dev, int32_t ntensors,
                         const mdemi_adamw_group* sched_dev, int32_t nsteps, int32_t ngroups,
                         int32_t* step_dev, int32_t* tensor_steps, const float* sumsq, float max_norm,
                         float grad_scale, int64_t nitems, void* workspace, void* stream);
/* The same two steps, also writing the RNE bf16 copy of every updated parameter t whose
 * param16_dev[t] (a device array of ntensors pointers, entries may be null) is set: the
 * bf16 operand its GEMMs read under bf16 storage (mdemi_gemm_bf16x), bit-identical to
 * mdemi_cast_bf16 of the new values -- no per-weight cast sweep in the next forward.
 * Replaces the per-step weight casts of autocast's bf16 weight cache
 * (depthformer_v8.py:46-75 under torch.autocast; configs[4]). */
int mdemi_adamw_step16(const mdemi_tensor_ref* tensors_dev, int32_t ntensors,
                       const mdemi_adamw_group* groups_host, int32_t ngroups,
                       const float* sumsq, float max_norm, float grad_scale, int32_t step,
                       int32_t* tensor_steps, int64_t nitems, void* const* param16_dev, void* workspace,
                       void* stream);
int mdemi_adamw_step_dev16(const mdemi_tensor_ref* tensors_dev, int32_t ntensors,
                           const mdemi_adamw_group* sched_dev, int32_t nsteps, int32_t ngroups,
                           int32_t* step_dev, int32_t* tensor_steps, const float* sumsq, float max_norm,
                           float grad_scale, int64_t nitems, void* const* param16_dev, void* workspace,
                           void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MDEMI_H */
