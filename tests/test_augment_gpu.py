"""GPU data pipeline (csrc/augment.hip through mdemi.dataset.GpuSampleTransform) against the
reference's own DepthDataset outputs (tests/golden/augment.npz) and, at the benchmark
sizes, against the oracle (oracle/augment.py, pinned to the reference and to Pillow by
tests/test_augment_oracle.py).

Tolerances: depth is bit-exact (integer geometry, one IEEE division); the image is
bit-exact up to powf (numpy/glibc vs the device's powf, ~1 ulp before the ImageNet
normalisation scales it by at most 1/0.224): |diff| <= 2e-6."""
import random

import numpy as np
import pytest
import torch

from golden_util import AUGMENT_CASES, GOLDEN, augment_inputs
from mdemi.dataset import DepthDataset, GpuSampleTransform, collate_raw, kb_crop_box
from oracle import augment as A

pytestmark = pytest.mark.gpu
IMG_ATOL = 2e-6


def _check(img, d, ref_img, ref_d):
    d = d.cpu().numpy()
    img = img.cpu().numpy()
    np.testing.assert_array_equal(d, ref_d)
    np.testing.assert_allclose(img, ref_img, rtol=0, atol=IMG_ATOL)


def _raw_batch(case, frame_kb):
    rgbs, deps = zip(*(augment_inputs(case, i) for i in range(case["n"])))
    if frame_kb:
        t, l = kb_crop_box(*case["raw"])
        rgbs = [r[t:t + 352, l:l + 1216] for r in rgbs]
        deps = [d[t:t + 352, l:l + 1216] for d in deps]
    return (torch.from_numpy(np.ascontiguousarray(np.stack(rgbs))),
            torch.from_numpy(np.ascontiguousarray(np.stack(deps)).view(np.int16)))


@pytest.mark.parametrize("name", sorted(AUGMENT_CASES))
def test_gpu_transform_matches_reference_dataset(name):
    from test_augment_oracle import _frame_hw, _transform
    case = AUGMENT_CASES[name]
    g = np.load(f"{GOLDEN}/augment.npz")
    tf = _transform(case)  # Pillow 12's I;16 nearest path, as the fixture ran
    rgb, dep = _raw_batch(case, case["data_type"] == "KITTI")
    params = [tf.draw(1, _frame_hw(case), random.Random(case["seed"] + i))[0] for i in range(case["n"])]
    img, d, _ = tf(rgb.cuda(), dep.cuda(), params)
    _check(img, d, g[f"{name}/image"], g[f"{name}/depth"])


@pytest.mark.parametrize("data_type", ["NYU", "KITTI"])
def test_gpu_transform_full_size_vs_oracle(data_type):
    """Benchmark sizes: NYU 480x640 frames -> 416x544 crops (the reference's commented
    alternative) and whole frames; KITTI 375x1242 raw -> KB crop -> 352x704 train crops
    (depth_dataset.py:52), Pillow 9.0.1's fixed-point nearest path; batch 4 from the host."""
    nyu = data_type == "NYU"
    case = dict(data_type=data_type, raw=(480, 640) if nyu else (375, 1242), seed=71 if nyu else 73,
                depth_max=20000 if nyu else 30000, n=4)
    frame = case["raw"] if nyu else (352, 1216)
    for crop in ([(416, 544), (480, 640)] if nyu else [(352, 704)]):
        tf = GpuSampleTransform(data_type, "train", crop, 2.5 if nyu else 1.0, 1000 if nyu else 256,
                                10.0 if nyu else 80.0, width_drop=(0.2, 4))
        rgb, dep = _raw_batch(case, not nyu)
        params = tf.draw(4, frame, random.Random(5))
        params[0]["angle"], params[1]["flip"] = 0.0, True  # unrotated copy path, a flipped sample
        params[2]["x"], params[2]["y"] = frame[1] - crop[1], frame[0] - crop[0]  # maximal crop offsets
        img, d, _ = tf(rgb, dep, params)  # host tensors: the transform uploads them
        for i, p in enumerate(params):
            r, dd = augment_inputs(case, i)
            ri, rd = A.sample(r, dd, p, data_type, "train", crop, tf.saving_factor, tf.clip_depth, nearest_fixed=True)
            _check(img[i], d[i], ri, rd)


def test_gpu_transform_kitti_test_mode():
    case = dict(data_type="KITTI", raw=(376, 1241), seed=79, depth_max=30000, n=2)
    tf = GpuSampleTransform("KITTI", "test", (376, 1241), None, 256, 80.0)
    rgb, dep = _raw_batch(case, True)
    img, d, params = tf(rgb.cuda(), dep.cuda())
    assert img.shape == (2, 3, 352, 1216) and d.shape == (2, 1, 352, 1216)
    for i in range(2):
        r, dd = augment_inputs(case, i)
        ri, rd = A.sample(r, dd, params[i], "KITTI", "test", (352, 1216), 256, 80.0)
        _check(img[i], d[i], ri, rd)


def test_dataset_decode_and_gpu_transform(tmp_path):
    """DepthDataset (host decode of PNG files, KB crop) -> collate_raw (pinned) -> the GPU
    transform, against the oracle on the same files."""
    from PIL import Image
    case = dict(data_type="KITTI", raw=(375, 1242), seed=83, depth_max=30000, n=2)
    (tmp_path / "raw").mkdir()
    (tmp_path / "gts").mkdir()
    lines = []
    for i in range(2):
        r, dd = augment_inputs(case, i)
        Image.fromarray(r).save(tmp_path / "raw" / f"i{i}.png")
        Image.fromarray(dd).save(tmp_path / "gts" / f"d{i}.png")
        lines.append(f"i{i}.png d{i}.png 721.5377\n")
    ds = DepthDataset(str(tmp_path), "KITTI", "train", filenames=lines)
    batch = collate_raw([ds[0], ds[1]], pin=True)
    assert batch["image"].shape == (2, 352, 1216, 3) and batch["focal"][0].item() == pytest.approx(721.5377)
    tf = ds.transform()
    img, d, params = tf(batch["image"], batch["depth"], rnd=random.Random(3))
    assert img.shape == (2, 3, 352, 704)
    for i in range(2):
        r, dd = augment_inputs(case, i)
        ri, rd = A.sample(r, dd, params[i], "KITTI", "train", (352, 704), 256, 80.0, nearest_fixed=True)
        _check(img[i], d[i], ri, rd)


def test_bad_arguments_raise():
    tf = GpuSampleTransform("NYU", "train", (64, 64), 2.5, 1000, 10.0)
    with pytest.raises(ValueError):
        tf(torch.zeros(1, 32, 32, 3, dtype=torch.uint8).cuda(), torch.zeros(1, 32, 32, dtype=torch.int16).cuda())
    with pytest.raises(ValueError):
        tf(torch.zeros(1, 80, 80, 3, dtype=torch.float32).cuda(), torch.zeros(1, 80, 80, dtype=torch.int16).cuda())
