"""Data pipeline: mirror of dataset/depth_dataset.py with the per-sample transform on the GPU.

The reference's ``DepthDataset.__getitem__`` (:166-236) decodes one sample with Pillow and
then crops, rotates, flips, colour-augments and normalises it in numpy on a DataLoader
worker.  Here the worker only decodes the files (``DepthDataset.__getitem__`` returns the
raw uint8 RGB and uint16 depth, KITTI already KB-cropped, :197-206), the batch is stacked
(``collate_raw``; pass ``DataLoader(pin_memory=True)`` so the main process's pin thread, not a
forked worker, pins it), and ``GpuSampleTransform`` runs everything after decoding as one
libmdemi sweep over the batch (``mdemi_augment``, csrc/augment.hip): the NYU valid-region
mask (:213-217), Pillow's rotate (:219-222), /255 and /saving_factor (:224-228),
random_crop (:238-248), the flip and colour augmentation (:250-280), hide_depth
(:282-284), ImageDepth2Tensor's normalisation (:287-311) and RandomMasking (:314-386).

The random draws stay on the host, in the reference's per-sample order (``draw``), so a
seeded ``random.Random`` yields the reference's parameters.  Constructor arguments,
attributes (height, width, degree, saving_factor, min/max/clip depth, do_kb_crop) and
ValueErrors follow ``DepthDataset.__init__`` (:13-161).
"""
from __future__ import annotations

import ctypes
import math
import os
import random
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _lib as L

_LIST_ROOT = os.path.join(".", "dataset", "train_test_inputs")  # the reference's relative list paths
_LISTS = {  # (data_type, mode) -> file list (depth_dataset.py:49-149)
    ("KITTI", "train"): "KITTI/kitti_eigen_train.txt", ("KITTI", "test"): "KITTI/kitti_eigen_test.txt",
    ("NYU", "train"): "NYU/nyu_train_36k.txt", ("NYU", "test"): "NYU/nyu_test.txt",
    ("ONLINE", "train"): "KITTI/kitti_benchmark_train.txt", ("ONLINE", "test"): "KITTI/kitti_benchmark_val.txt",
    ("ONLINE", "benchmark"): "KITTI/kitti_benchmark_test.txt",
}
NYU_FOCAL = 518.8579  # depth_dataset.py:172


def _config(data_type: str, mode: str, img_size):
    """(height, width, do_random_rotate, degree, min, max, saving_factor, do_kb_crop) of
    DepthDataset.__init__ (:46-154)."""
    if data_type in ("KITTI", "ONLINE"):
        if mode == "train":
            hw, rot, deg = (352, 704), True, 1.0
        else:
            hw, rot, deg = (376, 1241), False, None
        max_depth = 80.0 if data_type == "KITTI" else 88.0
        return (*(img_size or hw), rot, deg, 0.001, max_depth, 256, True)
    if mode == "train":
        return (*(img_size or (480, 640)), True, 2.5, 0.001, 10.0, 1000, False)
    return (*(img_size or (480, 640)), False, None, 0.001, 10.0, 1000, False)


def kb_crop_box(height: int, width: int) -> Tuple[int, int]:
    """(top, left) of the KB crop to 352 x 1216 (:201-206)."""
    return int(height - 352), int((width - 1216) / 2)


def rotate_matrix(angle: float, w: int, h: int) -> List[float]:
    """Pillow's Image.rotate inverse affine map (counter-clockwise `angle` degrees about the
    image centre, expand=False): the matrix ImagingTransformAffine receives."""
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


def _fix(v: float) -> int:  # Pillow Geometry.c FIX(): 16.16 fixed point
    return int(math.floor(v * 65536.0 + 0.5))


def fixed_matrix(m: List[float]) -> List[int]:
    """The 16.16 fixed-point coefficients of Pillow's affine_fixed for matrix m (nearest
    resampling of modes F and I): a0, a1, a2 (+half-pixel), a3, a4, a5 (+half-pixel)."""
    a, b, c, d, e, f = m
    return [_fix(a), _fix(b), _fix(c + a * 0.5 + b * 0.5), _fix(d), _fix(e), _fix(f + d * 0.5 + e * 0.5)]


def _fixed_ok(m, w, h) -> bool:  # Pillow check_fixed at (0, 0) and (w, h)
    a, b, c, d, e, f = m
    return all(abs(a * x + b * y + c) < 32768.0 and abs(d * x + e * y + f) < 32768.0 for x, y in ((0, 0), (w, h)))


class DepthDataset(torch.utils.data.Dataset):
    """Same constructor, attributes and errors as the reference's DepthDataset (:13-161);
    ``__getitem__`` returns the decoded sample (image uint8 (H,W,3), depth uint16 (H,W),
    KITTI/ONLINE KB-cropped) for the GPU transform instead of the finished tensors."""

    def __init__(self, data_path: str, data_type: str = "NYU", mode: str = "train",
                 img_size: Optional[Tuple[int, int]] = None, height_drop: Tuple[float, int] = (0.0, 0),
                 width_drop: Tuple[float, int] = (0.0, 0), clip_depth: Optional[float] = None,
                 use_right: bool = False, drop_edge: bool = False, list_root: str = _LIST_ROOT,
                 filenames: Optional[List[str]] = None):
        super().__init__()
        mode = mode.lower()
        if mode not in ("train", "test", "benchmark"):
            raise ValueError(f"DepthDataset mode {mode} is not supported.")
        data_type = data_type.upper()
        if data_type not in ("KITTI", "NYU", "ONLINE"):
            raise ValueError(f"DepthDataset data_type {data_type} is not supported.")
        if (mode == "benchmark") and (data_type != "ONLINE"):
            raise ValueError("Benchmark should only run with ONLINE data type.")
        if use_right:
            raise ValueError("DepthDataset currently do not support use_right=True option.")
        self.data_path, self.data_type, self.mode, self.use_right = data_path, data_type, mode, use_right
        (self.height, self.width, self.do_random_rotate, self.degree, self.min_depth, self.max_depth,
         self.saving_factor, self.do_kb_crop) = _config(data_type, mode, img_size)
        if data_type == "KITTI" or (data_type == "ONLINE" and mode == "train"):
            self.img_path, self.gt_path = os.path.join(data_path, "raw"), os.path.join(data_path, "gts")
        else:
            self.img_path = data_path
            self.gt_path = None if mode == "benchmark" else data_path
        self.clip_depth = self.max_depth if clip_depth is None else clip_depth
        self.height_drop, self.width_drop, self.drop_edge = height_drop, width_drop, drop_edge
        if drop_edge and min(height_drop[1], 1) == 0 and min(width_drop[1], 1) == 0:
            raise ValueError("If drop_edge is ON, you should use at least 1 drop_count.")
        if filenames is None:
            with open(os.path.join(list_root, _LISTS[(data_type, mode)]), "r") as f:
                filenames = list(f.readlines())
        self.filenames = filenames

    def __len__(self) -> int:
        return len(self.filenames)

    def __getitem__(self, idx: int) -> Dict:
        from PIL import Image
        path = self.filenames[idx].replace("\n", "").strip()
        focal = float(path.split()[2]) if self.data_type == "KITTI" else NYU_FOCAL
        if self.mode != "benchmark":
            ip, dp = (p[1:] if p.startswith("/") else p for p in path.split()[:2])
            image = np.asarray(Image.open(os.path.join(self.img_path, ip)), dtype=np.uint8)
            depth = np.asarray(Image.open(os.path.join(self.gt_path, dp))).astype(np.uint16)
        else:
            ip, dp = (path[1:] if path.startswith("/") else path), ""
            image = np.asarray(Image.open(os.path.join(self.img_path, ip)), dtype=np.uint8)
            depth = np.zeros(image.shape[:2], dtype=np.uint16)
        if self.do_kb_crop:
            if depth.shape != image.shape[:2]:
                raise ValueError(f"image {image.shape[:2]} and depth {depth.shape} sizes differ")
            top, left = kb_crop_box(*image.shape[:2])
            image, depth = image[top:top + 352, left:left + 1216], depth[top:top + 352, left:left + 1216]
        return {"image": np.ascontiguousarray(image[..., :3]), "depth": np.ascontiguousarray(depth),
                "focal": focal, "image_path": ip, "depth_path": dp}

    def transform(self) -> "GpuSampleTransform":
        return GpuSampleTransform(self.data_type, self.mode, (self.height, self.width),
                                  self.degree if self.do_random_rotate else None, self.saving_factor,
                                  self.clip_depth, self.height_drop, self.width_drop, self.drop_edge)


def collate_raw(samples: List[Dict], pin: bool = False) -> Dict:
    """Stack decoded samples into (B,H,W,3) uint8 / (B,H,W) uint16 host tensors.
    pin=True pins them here -- only in a process that may initialise HIP (not a forked
    DataLoader worker: use DataLoader(collate_fn=collate_raw, pin_memory=True) there)."""
    img = torch.from_numpy(np.stack([s["image"] for s in samples]))
    dep = torch.from_numpy(np.stack([s["depth"] for s in samples]).view(np.int16))
    if pin and torch.cuda.is_available():
        img, dep = img.pin_memory(), dep.pin_memory()
    return {"image": img, "depth": dep, "focal": torch.tensor([s["focal"] for s in samples]),
            "image_path": [s["image_path"] for s in samples], "depth_path": [s["depth_path"] for s in samples]}


class GpuSampleTransform:
    """Everything DepthDataset does after decoding, for a batch, on the GPU."""

    def __init__(self, data_type: str = "NYU", mode: str = "train", crop_hw: Tuple[int, int] = (480, 640),
                 degree: Optional[float] = 2.5, saving_factor: float = 1000, clip_depth: float = 10.0,
                 height_drop: Tuple[float, int] = (0.0, 0), width_drop: Tuple[float, int] = (0.0, 0),
                 drop_edge: bool = False, nearest_mode: str = "fixed"):
        self.data_type, self.mode = data_type.upper(), mode.lower()
        self.h, self.w = crop_hw
        self.degree, self.saving_factor, self.clip_depth = degree, float(saving_factor), float(clip_depth)
        self.height_drop, self.width_drop, self.drop_edge = height_drop, width_drop, drop_edge
        # NYU depth is rotated as mode "F" (:213-222) and, under Pillow 9.0.1 (the reference's
        # pinned version, output/.../requirements.txt), KITTI's 16-bit PNG depth opens as mode
        # "I": both take Pillow's 16.16 fixed-point nearest path.  nearest_mode="generic" is
        # the mode-I;16 path newer Pillow takes for the KITTI/ONLINE depth.
        if nearest_mode not in ("fixed", "generic"):
            raise ValueError(f"nearest_mode must be 'fixed' or 'generic', got {nearest_mode!r}")
        self.nearest_generic = nearest_mode == "generic" and self.data_type != "NYU"

    # -- host: the random draws, in depth_dataset.py's per-sample order
    def draw(self, batch: int, frame_hw: Tuple[int, int], rnd=random) -> List[Dict]:
        H, W = frame_hw
        out = []
        for _ in range(batch):
            p = {"angle": 0.0, "x": 0, "y": 0, "flip": False, "gamma": 1.0, "brightness": 1.0,
                 "colors": [1.0, 1.0, 1.0], "rows": [], "cols": []}
            if self.mode == "train":
                if self.degree:
                    p["angle"] = (rnd.random() - 0.5) * 2 * self.degree  # :220
                if (H, W) != (self.h, self.w):  # random_crop :241-245
                    if H < self.h or W < self.w:
                        raise ValueError(f"crop {self.h}x{self.w} larger than the frame {H}x{W}")
                    p["x"] = rnd.randint(0, W - self.w)
                    p["y"] = rnd.randint(0, H - self.h)
                p["flip"] = rnd.random() > 0.5  # :252
                p["gamma"] = rnd.uniform(0.9, 1.1)  # :264
                p["brightness"] = rnd.uniform(0.75, 1.25) if self.data_type == "NYU" else rnd.uniform(0.9, 1.1)
                p["colors"] = [rnd.uniform(0.9, 1.1) for _ in range(3)]  # :275-277
                p["rows"], p["cols"] = self._masking(rnd)
            out.append(p)
        return out

    def _masking(self, rnd):  # RandomMasking.__call__ :337-381 as spans
        h, w = self.h, self.w
        hr, hc = max(min(self.height_drop[0], 1.0), 0.0), max(self.height_drop[1], 0)
        wr, wc = max(min(self.width_drop[0], 1.0), 0.0), max(self.width_drop[1], 0)
        rows, cols = [], []
        if not self.drop_edge:
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
            hk, wk = int((h - 1) * (1.0 - hr)), int((w - 1) * (1.0 - wr))
            if min(hc, 1) > 0:
                n = rnd.randint(0, hk)
                s = rnd.randint(0, h - n)
                rows.append((1, s, s + n))
            if min(wc, 1) > 0:
                n = rnd.randint(0, wk)
                s = rnd.randint(0, w - n)
                cols.append((1, s, s + n))
        if len(rows) > L.AUG_MAX_SPANS or len(cols) > L.AUG_MAX_SPANS:
            raise ValueError(f"RandomMasking: at most {L.AUG_MAX_SPANS} drops per axis on the GPU path")
        return rows, cols

    def pack(self, params: List[Dict], frame_hw: Tuple[int, int], crop_hw: Tuple[int, int]) -> bytes:
        H, W = frame_hw
        h, w = crop_hw
        arr = (L.AugSample * len(params))()
        for s, p in zip(arr, params):
            rot = (p["angle"] % 360.0) != 0
            m = rotate_matrix(p["angle"], W, H) if rot else [1.0, 0.0, 0.0, 0.0, 1.0, 0.0]
            if rot and not self.nearest_generic and not _fixed_ok(m, W, H):
                raise ValueError("rotation outside Pillow's fixed-point range")
            s.affine[:] = m
            s.fixed[:] = fixed_matrix(m)
            s.rotate = int(rot)
            if not (0 <= p["x"] <= W - w and 0 <= p["y"] <= H - h):
                raise ValueError(f"crop offset ({p['y']}, {p['x']}) outside the {H}x{W} frame")
            s.crop_x, s.crop_y, s.flip = p["x"], p["y"], int(bool(p["flip"]))
            s.gamma, s.brightness = p["gamma"], p["brightness"]
            s.color[:] = list(p["colors"])
            s.n_rows, s.n_cols = len(p["rows"]), len(p["cols"])
            s.mask_keep = int(any(k == 1 for k, _, _ in p["rows"] + p["cols"]))
            for i, (_, a, b) in enumerate(p["rows"]):
                s.rows[i][0], s.rows[i][1] = a, b
            for i, (_, a, b) in enumerate(p["cols"]):
                s.cols[i][0], s.cols[i][1] = a, b
        return bytes(arr)

    # -- device: one sweep
    def __call__(self, image: torch.Tensor, depth: torch.Tensor, params: Optional[List[Dict]] = None,
                 rnd=random) -> Tuple[torch.Tensor, torch.Tensor, List[Dict]]:
        """image (B,H,W,3) uint8, depth (B,H,W) uint16/int16 (host or device; host batches are
        copied asynchronously) -> (image (B,3,h,w) fp32, depth (B,1,h,w) fp32, params)."""
        if image.dim() != 4 or image.shape[-1] != 3 or image.dtype != torch.uint8:
            raise ValueError(f"image must be (B,H,W,3) uint8, got {tuple(image.shape)} {image.dtype}")
        if depth.shape != image.shape[:3] or depth.element_size() != 2:
            raise ValueError(f"depth must be (B,H,W) 16-bit, got {tuple(depth.shape)} {depth.dtype}")
        B, H, W = image.shape[:3]
        h, w = (self.h, self.w) if self.mode == "train" else (H, W)  # test: no random_crop
        if not (h <= H and w <= W):
            raise ValueError(f"crop {h}x{w} larger than the frame {H}x{W}")
        dev = torch.device("cuda", torch.cuda.current_device())
        if params is None:
            params = self.draw(B, (H, W), rnd)
        tab = torch.frombuffer(bytearray(self.pack(params, (H, W), (h, w))), dtype=torch.uint8).to(dev)
        img_d = image.to(dev, non_blocking=True).contiguous()
        dep_d = depth.to(dev, non_blocking=True).contiguous()
        out_i = torch.empty(B, 3, h, w, device=dev)
        out_d = torch.empty(B, 1, h, w, device=dev)
        L.call("mdemi_augment", img_d.data_ptr(), dep_d.data_ptr(), B, H, W, 0, 0, H, W, h, w,
               tab.data_ptr(), int(self.data_type == "NYU" and self.mode == "train"), int(self.nearest_generic),
               int(self.mode == "train"), ctypes.c_float(self.saving_factor), ctypes.c_float(self.clip_depth),
               out_i.data_ptr(), out_d.data_ptr(), L.stream())
        return out_i, out_d, params
