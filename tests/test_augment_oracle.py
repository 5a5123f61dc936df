"""The data-pipeline oracle (oracle/augment.py) pinned two ways, on CPU:
* its restatement of Pillow's Image.rotate (bilinear RGB, nearest F / I / I;16) is
  bit-exact against Pillow itself on random images and angles;
* the whole sample transform, fed mdemi.dataset.GpuSampleTransform.draw's parameters for
  the seed the reference was run with, reproduces the reference's own DepthDataset
  outputs (tests/golden/augment.npz, tests/golden/make_golden_augment.py) bit-exactly."""
import random

import numpy as np
import pytest

from golden_util import AUGMENT_CASES, GOLDEN, augment_inputs
from mdemi.dataset import GpuSampleTransform, fixed_matrix, kb_crop_box, rotate_matrix
from oracle import augment as A

PIL = pytest.importorskip("PIL.Image")


@pytest.mark.parametrize("hw", [(480, 640), (352, 1216), (37, 53), (64, 64)])
def test_rotate_restatement_matches_pillow(hw):
    rng = np.random.default_rng(hw[0] * 7 + hw[1])
    H, W = hw
    for t in range(6):
        ang = [-2.5, 2.5, 0.0, 1e-7][t] if t < 4 else (rng.random() - 0.5) * 5
        rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        ref = np.asarray(PIL.fromarray(rgb).rotate(ang, resample=PIL.BILINEAR))
        np.testing.assert_array_equal(A.rotate_rgb_bilinear(rgb, ang), ref)
        f = rng.integers(0, 65535, (H, W)).astype(np.float32)  # mode F (NYU depth after the mask)
        np.testing.assert_array_equal(A.rotate_nearest(f, ang, fixed=True),
                                      np.asarray(PIL.fromarray(f).rotate(ang, resample=PIL.NEAREST)))
        i32 = rng.integers(0, 65535, (H, W)).astype(np.int32)  # mode I (16-bit PNG, Pillow 9.0.1)
        np.testing.assert_array_equal(A.rotate_nearest(i32, ang, fixed=True),
                                      np.asarray(PIL.fromarray(i32).rotate(ang, resample=PIL.NEAREST)))
        u16 = rng.integers(0, 65535, (H, W)).astype(np.uint16)  # mode I;16 (16-bit PNG, Pillow >= 10)
        im = PIL.fromarray(u16)
        assert im.mode == "I;16"
        np.testing.assert_array_equal(A.rotate_nearest(u16, ang, fixed=False),
                                      np.asarray(im.rotate(ang, resample=PIL.NEAREST)))


def test_host_matrices_match_oracle():
    for ang in (-2.5, -0.3, 0.7, 2.5, 359.0):
        m = rotate_matrix(ang, 640, 480)
        assert m == A.rotate_matrix(ang, 640, 480)
        a, b, c, d, e, f = m
        assert fixed_matrix(m) == [A._fix(a), A._fix(b), A._fix(c + a * 0.5 + b * 0.5), A._fix(d), A._fix(e),
                                   A._fix(f + d * 0.5 + e * 0.5)]


def _transform(case):
    h, w = case["img_size"] or case["raw"]
    deg = (2.5 if case["data_type"] == "NYU" else 1.0) if case["mode"] == "train" else None
    sf, clip = (1000, 10.0) if case["data_type"] == "NYU" else (256, 80.0)
    return GpuSampleTransform(case["data_type"], case["mode"], (h, w), deg, sf, clip,
                              tuple(case.get("height_drop", (0.0, 0))), tuple(case.get("width_drop", (0.0, 0))),
                              case.get("drop_edge", False), nearest_mode="generic")


def _frame_hw(case):
    return (352, 1216) if case["data_type"] == "KITTI" else case["raw"]


@pytest.mark.parametrize("name", sorted(AUGMENT_CASES))
def test_oracle_reproduces_reference_dataset(name):
    case = AUGMENT_CASES[name]
    g = np.load(f"{GOLDEN}/augment.npz")
    tf = _transform(case)
    sf, clip = tf.saving_factor, tf.clip_depth
    for i in range(case["n"]):
        rgb, dep = augment_inputs(case, i)
        p = tf.draw(1, _frame_hw(case), random.Random(case["seed"] + i))[0]
        img, d = A.sample(rgb, dep, p, case["data_type"], case["mode"], (tf.h, tf.w), sf, clip,
                          nearest_fixed=False)  # the fixture ran on Pillow 12 (16-bit PNG -> I;16)
        np.testing.assert_array_equal(d, g[f"{name}/depth"][i])
        np.testing.assert_array_equal(img, g[f"{name}/image"][i])


def test_kb_crop_box():
    assert kb_crop_box(375, 1242) == (23, 13)
    assert kb_crop_box(352, 1216) == (0, 0)


def test_aug_sample_struct_matches_header(tmp_path):
    """mdemi._lib.AugSample (ctypes) has the C layout of include/mdemi_ext.h's mdemi_aug_sample."""
    import ctypes
    import os
    import shutil
    import subprocess
    from mdemi import _lib as L
    if shutil.which("gcc") is None:
        pytest.skip("gcc absent")
    inc = os.path.dirname(L.HEADER_PATH)
    fields = [f[0] for f in L.AugSample._fields_]
    src = tmp_path / "probe.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "mdemi_ext.h"\nint main(void){\n'
                   + f'printf("%zu\\n", sizeof(mdemi_aug_sample));\n'
                   + "".join(f'printf("%zu\\n", offsetof(mdemi_aug_sample, {f}));\n' for f in fields) + "return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", inc, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got[0] == ctypes.sizeof(L.AugSample)
    assert got[1:] == [getattr(L.AugSample, f).offset for f in fields]
