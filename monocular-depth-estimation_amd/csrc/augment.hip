// Train/test sample transform of dataset/depth_dataset.py as one HBM sweep per batch
// (DepthDataset.__getitem__ :197-236 and the transforms it composes), from the decoded
// dataset files (RGB uint8 HWC, depth uint16) straight to the network's inputs:
//
//   KB crop (KITTI, :197-206) -> NYU valid-region mask (:213-217) -> Image.rotate
//   (image BILINEAR, depth NEAREST, :219-222) -> /255, /saving_factor (:224-228) ->
//   random crop (:238-248) -> horizontal flip (:252-254) -> gamma, brightness, colour,
//   clip (:262-280) -> hide_depth (:282-284) -> ImageNet normalise (:287-301) ->
//   RandomMasking (:314-386)
//
// One thread per output pixel; the per-sample random draws arrive as a table
// (mdemi_aug_sample) the host fills in the reference's draw order.  The rotation follows
// Pillow's geometry exactly (pinned to Pillow by tests/test_augment_oracle.py through
// oracle/augment.py): the bilinear image path evaluates the inverse affine map per pixel in
// double with no contraction and truncates to uint8; the nearest depth path steps 16.16
// fixed point (modes F and I) or floors the double map (mode I;16).
// Algorithmic bytes per output pixel: 3 (RGB) + 2 (depth) read, 12 + 4 written.
#include "common.h"
#include "mdemi_ext.h"

namespace mdemi {

__constant__ float AUG_MEAN[3] = {0.485f, 0.456f, 0.406f};  // depth_dataset.py:290
__constant__ float AUG_STD[3] = {0.229f, 0.224f, 0.225f};

__device__ __forceinline__ float span_mask(const mdemi_aug_sample& P, int y, int x) {
  bool in_row = false, in_col = false;
  for (int s = 0; s < P.n_rows; ++s) in_row |= (y >= P.rows[s][0] && y < P.rows[s][1]);
  for (int s = 0; s < P.n_cols; ++s) in_col |= (x >= P.cols[s][0] && x < P.cols[s][1]);
  if (P.mask_keep) return (in_row || in_col) ? 1.f : 0.f;  // drop_edge: zeros, keep spans set to 1
  return (in_row || in_col) ? 0.f : 1.f;
}

__global__ void __launch_bounds__(256) augment_kernel(const uint8_t* __restrict__ rgb, const uint16_t* __restrict__ dep,
                                                      int32_t B, int32_t H0, int32_t W0, int32_t top, int32_t left,
                                                      int32_t Hs, int32_t Ws, int32_t h, int32_t w,
                                                      const mdemi_aug_sample* __restrict__ params, int32_t nyu_mask,
                                                      int32_t nearest_generic, int32_t train, float saving_factor,
                                                      float clip_depth, float* __restrict__ img_out,
                                                      float* __restrict__ dep_out) {
#pragma clang fp contract(off)
  const int64_t total = (int64_t)B * h * w;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int32_t ox = (int32_t)(i % w);
  const int64_t t = i / w;
  const int32_t oy = (int32_t)(t % h);
  const int32_t b = (int32_t)(t / h);
  const mdemi_aug_sample& P = params[b];
  // pixel of the rotated frame (the KB-cropped image for KITTI) this output reads
  // (the host validates crop_x + w <= Ws, crop_y + h <= Hs; the clamp only keeps a bad
  // table from reading outside the source)
  const int32_t fx = min(max(P.crop_x + (P.flip ? w - 1 - ox : ox), 0), Ws - 1);
  const int32_t fy = min(max(P.crop_y + oy, 0), Hs - 1);
  const uint8_t* src = rgb + (int64_t)b * H0 * W0 * 3;
  const uint16_t* dsrc = dep + (int64_t)b * H0 * W0;
  auto texel = [&](int32_t y, int32_t x, int c) -> double {  // frame coords
    return (double)src[((int64_t)(top + y) * W0 + (left + x)) * 3 + c];
  };

  // ---- image: Pillow BILINEAR rotate (ImagingGenericTransform + bilinear_filter32RGB)
  float v[3];
  if (!P.rotate) {
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = (float)texel(fy, fx, c);
  } else {
    const double xo = (double)fx + 0.5, yo = (double)fy + 0.5;
    double xin = P.affine[0] * xo + P.affine[1] * yo + P.affine[2];
    double yin = P.affine[3] * xo + P.affine[4] * yo + P.affine[5];
    if (xin < 0.0 || xin >= (double)Ws || yin < 0.0 || yin >= (double)Hs) {
      v[0] = v[1] = v[2] = 0.f;
    } else {
      xin -= 0.5;
      yin -= 0.5;
      const double xf = floor(xin), yf = floor(yin);
      const double dx = xin - xf, dy = yin - yf;
      const int32_t x0 = (int32_t)xf, y0 = (int32_t)yf;
      const int32_t xa = min(max(x0, 0), Ws - 1), xb = min(max(x0 + 1, 0), Ws - 1);
      const int32_t ya = min(max(y0, 0), Hs - 1);
      const bool has_y1 = y0 + 1 >= 0 && y0 + 1 < Hs;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const double p0 = texel(ya, xa, c), p1 = texel(ya, xb, c);
        double v1 = p0 + (p1 - p0) * dx;
        double v2 = v1;
        if (has_y1) {
          const double q0 = texel(y0 + 1, xa, c), q1 = texel(y0 + 1, xb, c);
          v2 = q0 + (q1 - q0) * dx;
        }
        v1 = v1 + (v2 - v1) * dy;
        v[c] = (float)(uint8_t)v1;  // Pillow stores the double into UINT8 (truncation)
      }
    }
  }

  // ---- depth: Pillow NEAREST rotate of the (masked) depth plane
  int32_t sy = fy, sx = fx;
  if (P.rotate) {
    if (nearest_generic) {  // mode I;16: ImagingGenericTransform, COORD() floor
      const double xo = (double)fx + 0.5, yo = (double)fy + 0.5;
      const double xin = P.affine[0] * xo + P.affine[1] * yo + P.affine[2];
      const double yin = P.affine[3] * xo + P.affine[4] * yo + P.affine[5];
      sx = xin < 0.0 ? -1 : (int32_t)xin;
      sy = yin < 0.0 ? -1 : (int32_t)yin;
    } else {  // modes F / I: affine_fixed, 16.16 stepping
      const int64_t xx = (int64_t)P.fixed[2] + (int64_t)fy * P.fixed[1] + (int64_t)fx * P.fixed[0];
      const int64_t yy = (int64_t)P.fixed[5] + (int64_t)fy * P.fixed[4] + (int64_t)fx * P.fixed[3];
      sx = (int32_t)(xx >> 16);
      sy = (int32_t)(yy >> 16);
    }
  }
  float d = 0.f;
  if (sx >= 0 && sx < Ws && sy >= 0 && sy < Hs) {
    d = (float)dsrc[(int64_t)(top + sy) * W0 + (left + sx)];
    if (nyu_mask && !(sy >= 45 && sy < 472 && sx >= 43 && sx < 608)) d = 0.f;  // depth_mask[45:472, 43:608]
  }
  d = d / saving_factor;

  const float mk = train ? span_mask(P, oy, ox) : 1.f;
  if (train) {
    if (d > clip_depth) d = 0.f;  // hide_depth
  }
  const int64_t plane = (int64_t)h * w, pix = (int64_t)oy * w + ox;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float x = v[c] / 255.0f;
    if (train) {
      x = powf(x, P.gamma);
      x = x * P.brightness;
      x = x * P.color[c];
      x = fminf(fmaxf(x, 0.f), 1.f);
    }
    x = (x - AUG_MEAN[c]) / AUG_STD[c];
    img_out[((int64_t)b * 3 + c) * plane + pix] = train ? x * mk : x;
  }
  dep_out[(int64_t)b * plane + pix] = train ? d * mk : d;
}

}  // namespace mdemi

using namespace mdemi;

extern "C" int mdemi_augment(const uint8_t* rgb, const uint16_t* depth, int32_t B, int32_t H0, int32_t W0, int32_t top,
                             int32_t left, int32_t Hs, int32_t Ws, int32_t h, int32_t w,
                             const mdemi_aug_sample* params, int32_t nyu_mask, int32_t nearest_generic, int32_t train,
                             float saving_factor, float clip_depth, float* image, float* depth_out, void* stream) {
  MDEMI_REQUIRE(rgb && depth && params && image && depth_out, "augment: null pointer");
  MDEMI_REQUIRE(B > 0 && h > 0 && w > 0 && Hs > 0 && Ws > 0 && H0 > 0 && W0 > 0, "augment: bad sizes");
  MDEMI_REQUIRE(top >= 0 && left >= 0 && top + Hs <= H0 && left + Ws <= W0, "augment: frame outside the source image");
  MDEMI_REQUIRE(h <= Hs && w <= Ws, "augment: crop larger than the frame");
  MDEMI_REQUIRE(saving_factor > 0.f, "augment: saving_factor must be positive");
  const int64_t total = (int64_t)B * h * w;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL(augment_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, rgb, depth, B, H0, W0, top, left,
                     Hs, Ws, h, w, params, nyu_mask, nearest_generic, train, saving_factor, clip_depth, image,
                     depth_out);
  return check_launch("augment");
}
