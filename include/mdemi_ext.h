/*
 * mdemi_ext.h — second part of the libmdemi.so C ABI: the ops of the AdaBins
 * and Depthformer-v8 rows of the hot path and the
 * evaluation metrics (A19).  Same conventions as mdemi.h: fp32 device
 * pointers owned by the caller, channels-last activations, `stream` is a
 * hipStream_t passed as void*, 0 / negative MDEMI_E* return, scratch through
 * *_workspace_size() queries, no allocation, no synchronisation.
 *
 * Reference call sites are cited per entry point (paths relative to the
 * reference root).  EfficientNet-B5 itself is third-party
 * (rwightman/gen-efficientnet-pytorch `tf_efficientnet_b5_ap`, fetched by
 * torch.hub at unet_adaptive_bins.py:129 / depthformer_v8.py:89); its ops are
 * restated from that published architecture.
 */
#ifndef MDEMI_EXT_H
#define MDEMI_EXT_H

#include "mdemi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Depthwise KxK convolution over NHWC (groups == C, no bias): the MBConv /  */
/* DepthwiseSeparable conv_dw of EfficientNet-B5 (encoder walked at          */
/* unet_adaptive_bins.py:65-73, depthformer_v8.py:15-24).  w is the          */
/* reference layout [C][1][K][K].  pad_t / pad_l are the top / left padding; */
/* the bottom / right padding follows from OH / OW, which is how TF 'same'   */
/* padding (asymmetric for stride 2) is expressed.                           */
/* ------------------------------------------------------------------------ */
int mdemi_dwconv_fwd(const float* x, const float* w, float* y, int32_t N, int32_t H, int32_t W, int32_t C,
                     int32_t K, int32_t stride, int32_t pad_t, int32_t pad_l, int32_t OH, int32_t OW,
                     void* stream);
size_t mdemi_dwconv_bwd_workspace_size(int32_t N, int32_t C, int32_t K, int32_t OH, int32_t OW);
/* dx and/or dw may be NULL to skip that gradient; dw is overwritten. */
int mdemi_dwconv_bwd(const float* dy, const float* x, const float* w, float* dx, float* dw, int32_t N,
                     int32_t H, int32_t W, int32_t C, int32_t K, int32_t stride, int32_t pad_t, int32_t pad_l,
                     int32_t OH, int32_t OW, void* workspace, void* stream);

/* ------------------------------------------------------------------------ */
/* Per-(image, channel) spatial reductions and channel scaling over NHWC:    */
/* global average pooling and the gate of EfficientNet's SqueezeExcite,      */
/* torch.mean(aux, dim=1) (decoder_v8.py:161).                               */
/*   out[n][c] = scale * sum_p a[n][p][c] * (b ? b[n][p][c] : 1)             */
/*   y[n][p][c] = x[n][p][c] * g[n][c] + (add ? add[n][c] : 0)               */
/* ------------------------------------------------------------------------ */
size_t mdemi_spatial_reduce_workspace_size(int32_t N, int64_t HW, int32_t C);
int mdemi_spatial_reduce(const float* a, const float* b, float* out, int32_t N, int64_t HW, int32_t C,
                         float scale, void* workspace, void* stream);
int mdemi_chan_scale(const float* x, const float* g, const float* add, float* y, int32_t N, int64_t HW,
                     int32_t C, void* stream);
/* the same with y16 (may be NULL): the RNE bf16 copy of y (SqueezeExcite's output, read by
 * the MBConv projection conv as a bf16 GEMM operand under precision "bf16") */
int mdemi_chan_scale16(const float* x, const float* g, const float* add, float* y, void* y16, int32_t N,
                       int64_t HW, int32_t C, void* stream);

/* SqueezeExcite gate MLP (conv_reduce 1x1 + bias, swish, conv_expand 1x1 +  */
/* bias, sigmoid) on pooled [N][C]; wr [R][C], we [C][R].  hid receives the  */
/* pre-activation of conv_reduce [N][R] (saved for the backward).            */
int mdemi_se_gate_fwd(const float* pooled, const float* wr, const float* br, const float* we, const float* be,
                      float* hid, float* gate, int32_t N, int32_t C, int32_t R, void* stream);
/* dgate [N][C] -> dpooled_scale x dpooled [N][C] (1/HW: the gradient each position of the  */
/* mean receives) and the four parameter gradients (overwritten).                           */
size_t mdemi_se_gate_bwd_workspace_size(int32_t N, int32_t C, int32_t R);
int mdemi_se_gate_bwd(const float* pooled, const float* wr, const float* we, const float* hid,
                      const float* gate, const float* dgate, float* dpooled, float* dwr, float* dbr, float* dwe,
                      float* dbe, int32_t N, int32_t C, int32_t R, float dpooled_scale, void* workspace,
                      void* stream);

/* ------------------------------------------------------------------------ */
/* Row softmax with a pre-scale, y = softmax(scale * x) along the last dim:  */
/* attention probabilities of nn.TransformerEncoderLayer (layers.py:8-9),    */
/* PreNormLunaBlock (luna_layer.py:213-215, 244-246), SelfAttentionBlock     */
/* (self_attention.py:72-74).  Backward: dx = scale * y * (dy - <dy, y>).    */
/* ------------------------------------------------------------------------ */
int mdemi_softmax_fwd(const float* x, float* y, int64_t rows, int32_t cols, float scale, void* stream);
int mdemi_softmax_bwd(const float* y, const float* dy, float* dx, int64_t rows, int32_t cols, float scale,
                      int32_t accumulate, void* stream);
/* The same two, also writing the RNE bf16 copy of the result (y16 / dx16, optional): the
 * attention probabilities feed P.V and the score gradient feeds dQ / dK as bf16 GEMM operands
 * (luna_layer.py:202-250 and self_attention.py:61-80 under torch.autocast, configs[4]). */
int mdemi_softmax_fwd16(const float* x, float* y, void* y16, int64_t rows, int32_t cols, float scale, void* stream);
int mdemi_softmax_bwd16(const float* y, const float* dy, float* dx, void* dx16, int64_t rows, int32_t cols,
                        float scale, int32_t accumulate, void* stream);
/* Softmax whose bf16 copy y16 (required) is the DROPPED-OUT probabilities: y16 = RNE bf16 of
 * mdemi_dropout_dev(y, p, seed_dev, seed_add, offset) element for element (the mask index is
 * the element's flat position in y), while y keeps the softmax itself for the backward.  The
 * attention dropout of luna_layer.py:213-215,244-246 / self_attention.py:72-74 fused into the
 * probabilities sweep: P.V reads y16, with no dropout launch and no fp32 copy of dropout(P). */
int mdemi_softmax_fwd_drop16(const float* x, float* y, void* y16, int64_t rows, int32_t cols, float scale, float p,
                             const uint64_t* seed_dev, uint64_t seed_add, uint64_t offset, void* stream);

/* y = act(x) elementwise (MDEMI_ACT_* code): the standalone activations of
 * UpscaleConcatAct (layer_utils.py:121) and the bin regressor
 * (decoder_v8.py:82-90).  The backward is mdemi_elementwise(MDEMI_EW_ACT_BWD). */
int mdemi_act_fwd(const float* x, float* y, int64_t n, int32_t act, void* stream);

/* Inverted dropout with a counter-based mask: y = x * keep(seed, offset+i) / (1-p).
 * The mask is a pure function of (seed, offset, i), so the backward is the
 * same call on dy (nn.Dropout in layers.py:8, luna_layer.py:172-173,
 * feed_forward.py:26, decoder_v8.py:84,87).  p == 0 is a copy. */
int mdemi_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed, uint64_t offset, void* stream);
/* mdemi_dropout with the seed read from device memory (seed_dev[0] + seed_add):
 * the caller draws seed_dev on the GPU (torch's graph-safe Philox), so a
 * hipGraph-captured train step gets a fresh mask on every replay. */
int mdemi_dropout_dev(const float* x, float* y, int64_t n, float p, const uint64_t* seed_dev, uint64_t seed_add,
                      uint64_t offset, void* stream);
/* The same mask, also writing y16 (optional; n % 4 == 0, 16-B aligned x / y, 8-B aligned
 * y16): the RNE bf16 copy of y for a bf16 GEMM that reads it -- the dropout backward's
 * gradient feeding the linear before it (luna_layer.py:172-173 under torch.autocast). */
int mdemi_dropout_dev16(const float* x, float* y, void* y16, int64_t n, float p, const uint64_t* seed_dev,
                        uint64_t seed_add, uint64_t offset, void* stream);

/* ------------------------------------------------------------------------ */
/* Channels-last adaptive-bin head: logits [B][HW][K] (the 1x1 conv_out /    */
/* bin_predictor output, unet_adaptive_bins.py:88-91,97, decoder_v8.py:      */
/* 158-159), pred[b][p] = sum_k softmax(logits)[k] * centers[b][k]            */
/* (unet_adaptive_bins.py:107, depthformer_v8.py:73).  stats [B][HW][2] =    */
/* (max, 1/sum) for the backward.                                            */
/* ------------------------------------------------------------------------ */
int mdemi_binhead_nhwc_fwd(const float* logits, const float* centers, float* pred, float* stats, int32_t B,
                           int64_t HW, int32_t K, void* stream);
size_t mdemi_binhead_nhwc_bwd_workspace_size(int32_t B, int64_t HW, int32_t K);
int mdemi_binhead_nhwc_bwd(const float* logits, const float* centers, const float* pred, const float* stats,
                           const float* dpred, float* dlogits, float* dcenters, int32_t B, int64_t HW, int32_t K,
                           void* workspace, void* stream);

/* Bin widths -> edges -> centres (unet_adaptive_bins.py:99-105 with         */
/* miniViT.py:38-46; depthformer_v8.py:62-66 with decoder_v8.py:163-166):     */
/*   w = act(raw) (mode 0: relu(x)+0.1, 1: elu(x, 0.1)+0.1), wn = w / sum w,  */
/*   edges = cumsum(pad((max-min)*wn, (1,0), min)), centres = mid-points.    */
/* widths_n [B][K] (normalised widths, AdaBins' bin_widths_normed) and        */
/* edges [B][K+1] may be NULL.  Backward: dcenters (+ dedges, dwidths_n,    */
/* each may be NULL) -> draw.                                                */
#define MDEMI_BINS_RELU 0
#define MDEMI_BINS_ELU 1
int mdemi_bins_fwd(const float* raw, float* widths_n, float* edges, float* centers, int32_t B, int32_t K,
                   int32_t mode, float min_val, float max_val, void* stream);
int mdemi_bins_bwd(const float* raw, const float* dcenters, const float* dedges, const float* dwidths_n,
                   float* draw, int32_t B, int32_t K, int32_t mode, float min_val, float max_val, void* stream);

/* ------------------------------------------------------------------------ */
/* Layout helpers                                                            */
/* ------------------------------------------------------------------------ */
/* NCHW -> NHWC with the channel dim zero-padded to Cp >= C (the 3-channel    */
/* image feeding EfficientNet's conv_stem through the implicit-GEMM conv).   */
int mdemi_nchw_to_nhwc_pad(const float* x, float* y, int32_t N, int32_t C, int64_t HW, int32_t Cp, void* stream);
/* Input gradient of a stride == kernel conv (no padding) over NHWC, the
 * scatter of its im2col columns (mViT's 16x16/16 embedding_encoder,
 * layers.py:13-18): x[n][y][x][c] = cols[(n*OH + y/p)*OW + x/p][((y%p)*p + x%p)*C + c]
 * for y < OH*p, x < OW*p; other pixels (dropped by the floor) get 0. */
int mdemi_unpatchify_nhwc(const float* cols, float* x, int32_t N, int32_t H, int32_t W, int32_t C, int32_t p,
                          int32_t OH, int32_t OW, void* stream);
/* Adjoint of replicate padding by p (padding_mode="replicate",              */
/* layer_utils.py:18-22): dx[n][y][x] = sum of dxp over the padded positions */
/* that clamp to (y, x).  dxp is [N][H+2p][W+2p][C].                          */
int mdemi_pad_fold_replicate(const float* dxp, float* dx, int32_t N, int32_t H, int32_t W, int32_t C, int32_t p,
                             void* stream);

/* ------------------------------------------------------------------------ */
/* Evaluation metrics on the GPU (utils/depth_utils.py:4-54): per image,     */
/* over valid = crop rectangle [y0,y1) x [x0,x1) & gt > min_depth &          */
/* gt < max_depth, the 9 metrics of tcompute_errors in this order:           */
/*   a1, a2, a3, abs_rel, sq_rel, rmse, rmse_log, silog, log_10              */
/* plus the valid-pixel count: out [B][10] (fp64).  clamp_pred != 0 clamps   */
/* pred into [min_depth, max_depth] first.                                   */
/* ------------------------------------------------------------------------ */
size_t mdemi_depth_metrics_workspace_size(int32_t B, int32_t H, int32_t W);
int mdemi_depth_metrics(const float* pred, const float* gt, int32_t B, int32_t H, int32_t W, int32_t y0,
                        int32_t y1, int32_t x0, int32_t x1, float min_depth, float max_depth, int32_t clamp_pred,
                        double* out, void* workspace, void* stream);

/* ------------------------------------------------------------------------ */
/* Flip-eval (config eval.flip_eval): rows of W floats (an NCHW batch is     */
/* B*C*H rows).  flip_w: y[r][w] = x[r][W-1-w] (out of place).              */
/* flip_avg_w: y[r][w] = (a[r][w] + b[r][W-1-w]) / 2; y may alias a.        */
/* ------------------------------------------------------------------------ */
int mdemi_flip_w(const float* x, float* y, int64_t rows, int32_t W, void* stream);
int mdemi_flip_avg_w(const float* a, const float* b, float* y, int64_t rows, int32_t W, void* stream);

/* ------------------------------------------------------------------------ */
/* AdaBins bin-centre chamfer loss (cfg loss.chamfer_weight; upstream        */
/* BinsChamferLoss over pytorch3d chamfer_distance -- the reference's loss  */
/* module is absent, parity unpinned).  from_edges: edges [B][P+1] (AdaBins) */
/* else centres [B][P] (Depthformer v8); gt [B][HW]; targets              */
/* are gt >= thresh.  fwd writes the batch-mean loss (loss[0]) and          */
/* dloss/dcentres [B][P] (gcent); bwd: dedges = dloss[0] (device scalar) *   */
/* the centre gradients pushed onto both edges of each bin.                 */
/* ------------------------------------------------------------------------ */
size_t mdemi_bins_chamfer_workspace_size(int32_t B, int32_t P, int64_t HW);
int mdemi_bins_chamfer_fwd(const float* edges, const float* gt, int32_t B, int32_t P, int32_t from_edges, int64_t HW,
                           float thresh, float* loss, float* gcent, void* workspace, void* stream);
int mdemi_bins_chamfer_bwd(const float* gcent, const float* dloss, float* dedges, int32_t B, int32_t P,
                           int32_t from_edges, void* stream);

/* ------------------------------------------------------------------------ */
/* Conv weight re-layouts (reference [Cout][Cin][KH][KW] <-> GEMM operands): */
/* OHWI: out[co][ky][kx][c] = w[co][c][ky][kx]  (fwd, patch-conv dgrad)     */
/* OIHW: out[co][c][ky][kx] = w[co][ky][kx][c]  (wgrad -> parameter layout) */
/* DGRAD: out[ky][kx][co][c] = w[co][c][KH-1-ky][KW-1-kx] (input gradient)   */
/* Out of place; cout/cin/kh/kw always describe the conv.                   */
/* ------------------------------------------------------------------------ */
#define MDEMI_WL_OHWI 0
#define MDEMI_WL_OIHW 1
#define MDEMI_WL_DGRAD 2
int mdemi_conv_weight_layout(const float* w, float* out, int32_t cout, int32_t cin, int32_t kh, int32_t kw,
                             int32_t mode, void* stream);
/* The same re-layout also writing out16 (optional): the RNE bf16 copy of `out`, the operand a bf16
 * conv GEMM reads (bf16 storage, configs[4]) -- one sweep instead of the re-layout plus a cast of
 * the fresh re-laid-out weight every step (layer_utils.py:20-24 ConvBN under torch.autocast). */
int mdemi_conv_weight_layout16(const float* w, float* out, void* out16, int32_t cout, int32_t cin, int32_t kh,
                               int32_t kw, int32_t mode, void* stream);

/* ------------------------------------------------------------------------ */
/* Sample transform of dataset/depth_dataset.py (replaces DepthDataset.      */
/* __getitem__ :197-236 after file decoding, with random_crop :238-248,      */
/* train_preprocess/augment_image/hide_depth :250-284, ImageDepth2Tensor     */
/* :287-311 and RandomMasking :314-386) for a batch of decoded samples:      */
/* rgb [B][H0][W0][3] uint8, depth [B][H0][W0] uint16 -> image [B][3][h][w]  */
/* ImageNet-normalised fp32, depth [B][1][h][w] = raw / saving_factor.       */
/* The frame (top, left, Hs, Ws) is the KITTI KB crop or the whole image;   */
/* the rotation (Pillow's Image.rotate about the frame centre) and the crop */
/* act inside it.  params: B device entries drawn by the host in the        */
/* reference's order (mdemi/data.py).  nyu_mask applies depth_mask           */
/* [45:472, 43:608] before the rotation; nearest_generic selects Pillow's    */
/* I;16 nearest path (else the 16.16 fixed-point path of modes F and I).     */
/* train = 0 is the test transform (no clip, hide_depth or masking).         */
/* ------------------------------------------------------------------------ */
#define MDEMI_AUG_MAX_SPANS 8
typedef struct {
  double affine[6];  /* Image.rotate's inverse map (x, y) -> source, in double     */
  int32_t fixed[6];  /* the same map in Pillow's 16.16 fixed point (affine_fixed)  */
  int32_t rotate;    /* 0: angle % 360 == 0 (Pillow returns a copy)                */
  int32_t crop_x, crop_y, flip;
  float gamma, brightness, color[3];
  int32_t n_rows, n_cols, mask_keep; /* RandomMasking spans; mask_keep: drop_edge */
  int32_t rows[MDEMI_AUG_MAX_SPANS][2];
  int32_t cols[MDEMI_AUG_MAX_SPANS][2];
} mdemi_aug_sample;
int mdemi_augment(const uint8_t* rgb, const uint16_t* depth, int32_t B, int32_t H0, int32_t W0, int32_t top,
                  int32_t left, int32_t Hs, int32_t Ws, int32_t h, int32_t w, const mdemi_aug_sample* params,
                  int32_t nyu_mask, int32_t nearest_generic, int32_t train, float saving_factor, float clip_depth,
                  float* image, float* depth_out, void* stream);

/* ------------------------------------------------------------------------ */
/* ODA2 ordered-swin2 (model/ODA2)                          */
/* ------------------------------------------------------------------------ */
/* Window shuffle of PreNormOrderedSwinSA (oda2_red_order_swin2_decoder.py:  */
/* 83-85,103,126-131): roll by -shift + window_partition as one gather       */
/* (inverse = 0): dst row r = ((n*nWh + wy)*nWw + wx)*ws^2 + ty*ws + tx       */
/* takes src[n][(wy*ws+ty+shift) % H][(wx*ws+tx+shift) % W]; inverse = 1 is  */
/* the scatter back (window_reverse + roll by +shift), optionally + add (the */
/* residual `out + identity`, natural layout).  H, W multiples of ws.         */
int mdemi_window_shuffle(const float* src, float* dst, const float* add, int32_t N, int32_t H, int32_t W,
                         int32_t C, int32_t ws, int32_t shift, int32_t inverse, void* stream);
/* the same gather for the int32 depth-index map [N][H][W] (:85,88) */
int mdemi_window_shuffle_i32(const int32_t* src, int32_t* dst, int32_t N, int32_t H, int32_t W, int32_t ws,
                             int32_t shift, void* stream);
/* Ordered window softmax (:87-92,116-119): S, P are [nwin][heads][T][T]     */
/* (T = ws^2 = 64 or 256), idx the window-major depth indices [nwin][T],     */
/* table the depth_embedding [2*num_emb-1][heads] (NULL: bias_type "none").  */
/*   P[w][h][i][j] = softmax_j(scale*S + table[idx_i - idx_j + num_emb-1][h]) */
/* S == P is allowed.  Backward: dS = scale * P o (dP - rowsum(P o dP)) and, */
/* when d_table != NULL, d_table[k][h] = sum of P o (dP - ...) over the     */
/* entries whose relative index is k (overwritten).                          */
int mdemi_ordered_softmax_fwd(const float* S, float* P, const int32_t* idx, const float* table, int32_t nwin,
                              int32_t heads, int32_t T, int32_t num_emb, float scale, void* stream);
size_t mdemi_ordered_softmax_bwd_workspace_size(int32_t nwin, int32_t heads, int32_t num_emb);
int mdemi_ordered_softmax_bwd(const float* P, const float* dP, float* dS, const int32_t* idx, float* d_table,
                              int32_t nwin, int32_t heads, int32_t T, int32_t num_emb, float scale, void* workspace,
                              void* stream);
/* nn.GLU(dim=-1) (oda2_red_order_reg_decoder.py:61,78): x [M][2F] ->        */
/* y [M][F] = x[:, :F] * sigmoid(x[:, F:]); bwd writes dx [M][2F].  F % 4 == 0 */
int mdemi_glu_fwd(const float* x, float* y, int64_t M, int32_t F, void* stream);
int mdemi_glu_bwd(const float* x, const float* dy, float* dx, int64_t M, int32_t F, void* stream);
/* Replicate padding / cropping as one clamp-gather over NHWC (the reference */
/* pads with F.pad(mode="replicate"): oda2_swin_transformer.py:258,327,491,  */
/* and the depthwise conv's padding_mode, oda2_red_order_reg_decoder.py:65): */
/*   y[n][oy][ox] = x[n][clamp(oy-pt, 0, H-1)][clamp(ox-pl, 0, W-1)], y is   */
/* [N][OH][OW][C].  inverse = 1 is the adjoint: x is the [N][OH][OW][C]       */
/* gradient, y the [N][H][W][C] sum over the positions that clamp to each   */
/* pixel.  An NCHW image is the NHWC map [N*C][H][W][1].                      */
int mdemi_pad_replicate(const float* x, float* y, int32_t N, int32_t H, int32_t W, int32_t C, int32_t OH,
                        int32_t OW, int32_t pt, int32_t pl, int32_t inverse, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MDEMI_EXT_H */
