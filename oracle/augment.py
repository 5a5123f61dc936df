"""CPU restatement of the train-time sample transform of dataset/depth_dataset.py
(DepthDataset.__getitem__ :197-236, random_crop :238-248, train_preprocess :250-260,
augment_image :262-280, hide_depth :282-284, ImageDepth2Tensor :287-311,
RandomMasking :314-386).  TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.

The reference rotates with Pillow (Image.rotate, :221-222).  Pillow's geometry is
restated here in numpy float64 (rotate_matrix / rotate_rgb_bilinear /
rotate_nearest) and pinned to Pillow itself, which is importable here:
tests/test_augment_oracle.py checks every restated rotation bit-exact against
PIL.Image.rotate on random images and angles, and the whole sample transform against
a Pillow + numpy pipeline written the way depth_dataset.py writes it.

Pillow paths (libImaging/Geometry.c, Pillow 12.2.0 as installed):
  * RGB + BILINEAR -> ImagingGenericTransform: per output pixel, the source point is
    a * (x + 0.5) + b * (y + 0.5) + c in double; the pixel is filled with 0 unless
    0 <= xin < W and 0 <= yin < H; then xin -= 0.5, yin -= 0.5, x0 = floor, the
    2x2 neighbours are clamped to the image (the lower row only if it exists), and
    the double result of the two-step lerp is truncated to uint8.
  * F (NYU depth after the valid-region mask) + NEAREST -> ImagingTransformAffine's
    16.16 fixed-point stepping (affine_fixed) when the matrix passes its range check.
  * I;16 (KITTI depth) + NEAREST -> ImagingGenericTransform with floor coordinates.
"""
import math

import numpy as np

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)  # depth_dataset.py:290
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def rotate_matrix(angle, w, h):
    """Image.rotate's inverse affine matrix (a, b, c, d, e, f) for a counter-clockwise
    rotation by `angle` degrees about the image centre (expand=False, no translate)."""
    angle = angle % 360.0
    ang = -math.radians(angle)
    m = [round(math.cos(ang), 15), round(math.sin(ang), 15), 0.0,
         round(-math.sin(ang), 15), round(math.cos(ang), 15), 0.0]
    cx, cy = w / 2, h / 2
    a, b, c, d, e, f = m
    m[2], m[5] = a * -cx + b * -cy + c, d * -cx + e * -cy + f
    m[2] += cx
    m[5] += cy
    return m


def _src_points(m, w, h):
    x = np.arange(w, dtype=np.float64)[None, :] + 0.5
    y = np.arange(h, dtype=np.float64)[:, None] + 0.5
    a, b, c, d, e, f = m
    return a * x + b * y + c, d * x + e * y + f


def rotate_rgb_bilinear(img, angle):
    """Image.fromarray(img (H,W,3) uint8).rotate(angle, resample=BILINEAR)."""
    h, w = img.shape[:2]
    if angle % 360.0 == 0:
        return img.copy()
    m = rotate_matrix(angle, w, h)
    xin, yin = _src_points(m, w, h)
    inside = (xin >= 0.0) & (xin < w) & (yin >= 0.0) & (yin < h)
    xs, ys = xin - 0.5, yin - 0.5
    x0, y0 = np.floor(xs), np.floor(ys)
    dx, dy = xs - x0, ys - y0
    x0 = x0.astype(np.int64)
    y0 = y0.astype(np.int64)
    xa, xb = np.clip(x0, 0, w - 1), np.clip(x0 + 1, 0, w - 1)
    ya = np.clip(y0, 0, h - 1)
    has_y1 = (y0 + 1 >= 0) & (y0 + 1 < h)
    yb = np.where(has_y1, np.clip(y0 + 1, 0, h - 1), ya)
    src = img.astype(np.float64)
    out = np.zeros_like(img)
    for ch in range(img.shape[2]):
        p = src[..., ch]
        v1 = p[ya, xa] + (p[ya, xb] - p[ya, xa]) * dx
        v2 = p[yb, xa] + (p[yb, xb] - p[yb, xa]) * dx
        v2 = np.where(has_y1, v2, v1)
        v = v1 + (v2 - v1) * dy
        out[..., ch] = np.where(inside, np.trunc(v), 0).astype(np.uint8)
    return out


def _fix(v):  # Geometry.c FIX(): 16.16 fixed point, round half up
    return int(math.floor(v * 65536.0 + 0.5))


def nearest_index_fixed(m, w, h):
    """Source (yi, xi) per output pixel of affine_fixed (mode F / 8-bit NEAREST)."""
    a, b, c, d, e, f = m
    a0, a1, a3, a4 = _fix(a), _fix(b), _fix(d), _fix(e)
    a2 = _fix(c + a * 0.5 + b * 0.5)
    a5 = _fix(f + d * 0.5 + e * 0.5)
    x = np.arange(w, dtype=np.int64)[None, :]
    y = np.arange(h, dtype=np.int64)[:, None]
    xx = a2 + y * a1 + x * a0
    yy = a5 + y * a4 + x * a3
    return yy >> 16, xx >> 16


def nearest_index_generic(m, w, h):
    """Source (yi, xi) per output pixel of ImagingGenericTransform + nearest (I;16)."""
    xin, yin = _src_points(m, w, h)
    xi = np.where(xin < 0.0, -1, np.floor(xin)).astype(np.int64)
    yi = np.where(yin < 0.0, -1, np.floor(yin)).astype(np.int64)
    return yi, xi


def fixed_path_ok(m, w, h):
    """affine_fixed's range check (check_fixed at (0,0) and (w,h))."""
    a, b, c, d, e, f = m

    def ok(x, y):
        return (abs(a * x + b * y + c) < 32768.0) and (abs(d * x + e * y + f) < 32768.0)
    return ok(0, 0) and ok(w, h)


def rotate_nearest(arr, angle, fixed):
    """Image.fromarray(arr (H,W)).rotate(angle, resample=NEAREST): fixed=True for mode F,
    False for mode I;16."""
    h, w = arr.shape
    if angle % 360.0 == 0:
        return arr.copy()
    m = rotate_matrix(angle, w, h)
    yi, xi = nearest_index_fixed(m, w, h) if fixed else nearest_index_generic(m, w, h)
    ok = (xi >= 0) & (xi < w) & (yi >= 0) & (yi < h)
    return np.where(ok, arr[np.clip(yi, 0, h - 1), np.clip(xi, 0, w - 1)], 0).astype(arr.dtype)


def draw_params(rnd, data_type, src_hw, crop_hw, degree, masking=((0.0, 0), (0.0, 0), False)):
    """The per-sample random draws of __getitem__ in the reference's order, from a
    `random.Random`-like `rnd`: rotation angle (:220), crop x, y (:244-245), flip (:252),
    gamma, brightness, 3 colour gains (:264-277), then RandomMasking (:350-381)."""
    H, W = src_hw
    h, w = crop_hw
    p = {"angle": (rnd.random() - 0.5) * 2 * degree if degree else 0.0}
    if (H, W) != (h, w):
        p["x"] = rnd.randint(0, W - w)
        p["y"] = rnd.randint(0, H - h)
    else:
        p["x"] = p["y"] = 0
    p["flip"] = rnd.random() > 0.5
    p["gamma"] = rnd.uniform(0.9, 1.1)
    p["brightness"] = rnd.uniform(0.75, 1.25) if data_type == "NYU" else rnd.uniform(0.9, 1.1)
    p["colors"] = [rnd.uniform(0.9, 1.1) for _ in range(3)]
    p["rows"], p["cols"] = random_masking_spans(rnd, h, w, *masking)
    return p


def random_masking_spans(rnd, h, w, height_drop=(0.0, 0), width_drop=(0.0, 0), drop_edge=False):
    """RandomMasking (:314-386) as (kind, start, end) spans; kind 0 zeroes [start, end),
    kind 1 (drop_edge) keeps only [start, end) of an all-zero mask."""
    hr, hc = max(min(height_drop[0], 1.0), 0.0), max(height_drop[1], 0)
    wr, wc = max(min(width_drop[0], 1.0), 0.0), max(width_drop[1], 0)
    rows, cols = [], []
    if not drop_edge:
        hmax, wmax = int((h - 1) * hr), int((w - 1) * wr)
        for _ in range(hc):
            n = rnd.randint(0, hmax)
            s = rnd.randint(0, h - n)
            rows.append((0, s, s + n))
        for _ in range(wc):
            n = rnd.randint(0, wmax)
            s = rnd.randint(0, w - n)
            cols.append((0, s, s + n))
    else:
        hc, wc = min(hc, 1), min(wc, 1)
        if hc == 0 and wc == 0:
            raise ValueError("If drop_edge is ON, you should use at least 1 drop_count.")
        hk, wk = int((h - 1) * (1.0 - hr)), int((w - 1) * (1.0 - wr))
        if hc > 0:
            n = rnd.randint(0, hk)
            s = rnd.randint(0, h - n)
            rows.append((1, s, s + n))
        if wc > 0:
            n = rnd.randint(0, wk)
            s = rnd.randint(0, w - n)
            cols.append((1, s, s + n))
    return rows, cols


def masking_plane(h, w, rows, cols):
    if any(k == 1 for k, _, _ in rows + cols):
        m = np.zeros((h, w), np.float32)
        for _, s, e in rows:
            m[s:e, :] = 1
        for _, s, e in cols:
            m[:, s:e] = 1
        return m
    m = np.ones((h, w), np.float32)
    for _, s, e in rows:
        m[s:e, :] = 0
    for _, s, e in cols:
        m[:, s:e] = 0
    return m


def sample(rgb, depth_raw, p, data_type, mode, crop_hw, saving_factor, clip_depth, nearest_fixed=True):
    """One sample: rgb (H0,W0,3) uint8, depth_raw (H0,W0) uint16 as decoded from the dataset
    files -> image (3,h,w) float32 normalised, depth (1,h,w) float32.  The KITTI KB crop
    (:197-206) is applied here when data_type is KITTI/ONLINE.  nearest_fixed: Pillow's
    nearest path for the KITTI depth (True: mode I, Pillow 9.0.1; False: mode I;16)."""
    if data_type in ("KITTI", "ONLINE"):
        H0, W0 = rgb.shape[:2]
        top, left = int(H0 - 352), int((W0 - 1216) / 2)
        rgb = rgb[top:top + 352, left:left + 1216]
        depth_raw = depth_raw[top:top + 352, left:left + 1216]
    if mode != "train":
        img = (rgb.astype(np.float32) / np.float32(255.0)).transpose(2, 0, 1)
        d = (depth_raw.astype(np.float32) / np.float32(saving_factor))[None]
        return ((img - MEAN[:, None, None]) / STD[:, None, None]).astype(np.float32), d.astype(np.float32)
    if data_type == "NYU":
        d = depth_raw.astype(np.float32)
        mask = np.zeros_like(d)
        mask[45:472, 43:608] = 1
        d = d * mask
        d = rotate_nearest(d, p["angle"], fixed=True)
    else:
        d = rotate_nearest(depth_raw, p["angle"], fixed=nearest_fixed).astype(np.float32)
    img = rotate_rgb_bilinear(rgb, p["angle"])
    img = img.astype(np.float32) / np.float32(255.0)
    d = (d / np.float32(saving_factor))[..., None]
    h, w = crop_hw
    img = img[p["y"]:p["y"] + h, p["x"]:p["x"] + w, :]
    d = d[p["y"]:p["y"] + h, p["x"]:p["x"] + w, :]
    if p["flip"]:
        img = img[:, ::-1, :].copy()
        d = d[:, ::-1, :].copy()
    img = img ** np.float32(p["gamma"])
    img = img * np.float32(p["brightness"])
    for ch in range(3):
        img[:, :, ch] *= np.float32(p["colors"][ch])
    img = np.clip(img, 0, 1)
    d = d.copy()
    d[d > np.float32(clip_depth)] = 0.0
    img = (img.transpose(2, 0, 1) - MEAN[:, None, None]) / STD[:, None, None]
    d = d.transpose(2, 0, 1)
    mk = masking_plane(h, w, p["rows"], p["cols"])
    return (img * mk).astype(np.float32), (d * mk).astype(np.float32)
