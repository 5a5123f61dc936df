"""Shared helpers for the golden fixtures (tests/golden/*.npz, written by
tests/golden/make_golden.py from the reference itself)."""
import json
import os
from collections import OrderedDict

import numpy as np
import torch

from oracle.newcrfs import relative_position_index
from oracle.weights import closed_form_fill, rng_array, rng_fill

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class Golden:
    def __init__(self, name):
        self.name = name
        self.d = np.load(os.path.join(GOLDEN, name + ".npz"))
        self.spec = json.loads(str(self.d["spec"]))
        self.fill = tuple(float(x) for x in self.d["fill"])
        self.fill_mode = str(self.d["fillmode"]) if "fillmode" in self.d else "closed_form"

    def keys(self, prefix):
        return [k[len(prefix):] for k in self.d.keys() if k.startswith(prefix)]

    def params(self, dtype=torch.float64):
        """Reference state_dict rebuilt from its spec + the closed-form fill."""
        P = OrderedDict()
        for name, shape, dt in self.spec:
            if dt.startswith("float"):
                P[name] = torch.zeros(shape, dtype=torch.float64)
            elif name.endswith("relative_position_index"):
                P[name] = relative_position_index(int(round(shape[0] ** 0.5)))
            else:
                P[name] = torch.zeros(shape, dtype=torch.int64)
        if self.fill_mode == "rng":
            rng_fill(P, seed=int(self.fill[0]), scale=self.fill[1])
        else:
            closed_form_fill(P, seed=self.fill[0], scale=self.fill[1])
        for k, v in P.items():
            if torch.is_floating_point(v):
                P[k] = v.to(dtype)
        return P

    def input(self, name, dtype=torch.float64):
        shape = tuple(int(x) for x in self.d[f"inshape/{name}"])
        return torch.from_numpy(rng_array(shape, int(self.d[f"inseed/{name}"]))).to(dtype)

    def input_names(self):
        return self.keys("inshape/")

    def dy(self, out_name, shape, dtype=torch.float64):
        return torch.from_numpy(rng_array(tuple(shape), int(self.d[f"dyseed/{out_name}"]))).to(dtype)

    def has(self, key):
        return key in self.d or ("sub/" + key) in self.d

    def check(self, key, value, rtol, atol=0.0):
        """Compare `value` with the stored array (full, or subsample + sums)."""
        v = value.detach().double().cpu().numpy().reshape(-1)
        if key in self.d:
            ref = self.d[key].astype(np.float64).reshape(-1)
            _assert_close(v, ref, rtol, atol, key)
        else:
            step = int(self.d["substep/" + key])
            ref = self.d["sub/" + key].astype(np.float64)
            _assert_close(v[::step], ref, rtol, atol, key)
            s = self.d["sum/" + key]
            got = np.array([v.sum(), (v * v).sum()])
            scale = np.sqrt(s[1] * v.size) + 1e-30
            assert abs(got[0] - s[0]) <= rtol * scale + atol * v.size, f"{key}: sum {got[0]} vs {s[0]}"
            assert abs(got[1] - s[1]) <= 2 * rtol * s[1] + 1e-30, f"{key}: sumsq {got[1]} vs {s[1]}"


def _assert_close(v, ref, rtol, atol, key):
    assert v.shape == ref.shape, f"{key}: shape {v.shape} vs {ref.shape}"
    err = np.abs(v - ref).max() if v.size else 0.0
    mag = np.abs(ref).max() if ref.size else 0.0
    assert err <= atol + rtol * mag, f"{key}: max|diff|={err:.3e} vs max|ref|={mag:.3e} (rtol={rtol})"


def spec_of(module):
    return [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in module.state_dict().items()]


# ---- dataset/depth_dataset.py fixtures (tests/golden/make_golden_augment.py -> augment.npz)
AUGMENT_CASES = {
    # NYU train: valid-region mask, rotate +-2.5 deg, random 64x96 crop of the 480x640 frame
    "nyu_train": dict(data_type="NYU", mode="train", raw=(480, 640), img_size=(64, 96), n=3, seed=11,
                      depth_max=20000),
    # KITTI train: KB crop of a 375x1242 frame, rotate +-1 deg, random 64x160 crop
    "kitti_train": dict(data_type="KITTI", mode="train", raw=(375, 1242), img_size=(64, 160), n=2, seed=23,
                        depth_max=30000),
    # RandomMasking: four width drops of up to 20 % and one height drop
    "nyu_train_masking": dict(data_type="NYU", mode="train", raw=(480, 640), img_size=(48, 64), n=2, seed=37,
                              depth_max=20000, height_drop=(0.3, 1), width_drop=(0.2, 4)),
    # drop_edge: keep one row band and one column band
    "nyu_train_drop_edge": dict(data_type="NYU", mode="train", raw=(480, 640), img_size=(48, 64), n=2, seed=41,
                                depth_max=20000, height_drop=(0.5, 1), width_drop=(0.5, 1), drop_edge=True),
    # NYU test: no augmentation, the whole (small) image
    "nyu_test": dict(data_type="NYU", mode="test", raw=(40, 56), img_size=None, n=2, seed=53, depth_max=20000),
}


def augment_inputs(case, i):
    """The decoded files of sample i of an AUGMENT_CASES case: RGB uint8 noise and uint16
    depth with ~10 % zeros (invalid pixels)."""
    rng = np.random.default_rng(case["seed"] * 1000 + i)
    H, W = case["raw"]
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    dep = rng.integers(1, case["depth_max"], (H, W)).astype(np.uint16)
    dep[rng.random((H, W)) < 0.1] = 0
    return rgb, dep
