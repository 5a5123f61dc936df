"""Generate tests/golden/augment.npz from the reference's own DepthDataset.

Runs dataset/depth_dataset.py from /root/reference (the reference is read, never copied;
only its outputs are stored) on synthetic decoded files written to a temporary directory:
torchvision is absent here, so the harness stubs torchvision.transforms.{Compose,Normalize}
(Normalize restated as torchvision.transforms.functional.normalize: (x - mean) / std per
channel).  For each case the global `random` is seeded, __getitem__ runs, and the finished
image / depth tensors are stored with the seed; the inputs are regenerated from
numpy.random.default_rng(seed) by tests/golden_util.augment_inputs.  The tests replay the
same seed through mdemi.dataset.GpuSampleTransform.draw (random.Random(seed)).

    python tests/golden/make_golden_augment.py      (needs /root/reference)
"""
import os
import random
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from golden_util import AUGMENT_CASES, augment_inputs  # noqa: E402

REF = "/root/reference"


def _stub_torchvision():
    tv = types.ModuleType("torchvision")
    tr = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, ts):
            self.ts = ts

        def __call__(self, x):
            for t in self.ts:
                x = t(x)
            return x

    class Normalize:
        def __init__(self, mean, std):
            self.mean, self.std = mean, std

        def __call__(self, t):
            m = torch.as_tensor(self.mean, dtype=t.dtype)[:, None, None]
            s = torch.as_tensor(self.std, dtype=t.dtype)[:, None, None]
            return t.sub(m).div(s)

    tr.Compose, tr.Normalize = Compose, Normalize
    tv.transforms = tr
    sys.modules["torchvision"], sys.modules["torchvision.transforms"] = tv, tr


def main():
    from PIL import Image
    _stub_torchvision()
    sys.path.insert(0, REF)
    from dataset.depth_dataset import DepthDataset  # the reference module
    out = {}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(REF)  # DepthDataset opens its file lists relative to the working directory
        try:
            for name, case in AUGMENT_CASES.items():
                root = os.path.join(tmp, name)
                sub = os.path.join(root, "raw") if case["data_type"] == "KITTI" else root
                gts = os.path.join(root, "gts") if case["data_type"] == "KITTI" else root
                os.makedirs(sub, exist_ok=True)
                os.makedirs(gts, exist_ok=True)
                lines = []
                for i in range(case["n"]):
                    rgb, dep = augment_inputs(case, i)
                    Image.fromarray(rgb).save(os.path.join(sub, f"img{i}.png"))
                    Image.fromarray(dep).save(os.path.join(gts, f"dep{i}.png"))
                    lines.append(f"/img{i}.png /dep{i}.png 721.5377\n")
                ds = DepthDataset(root, data_type=case["data_type"], mode=case["mode"],
                                  img_size=case.get("img_size"), height_drop=tuple(case.get("height_drop", (0.0, 0))),
                                  width_drop=tuple(case.get("width_drop", (0.0, 0))),
                                  drop_edge=case.get("drop_edge", False))
                ds.filenames = lines
                imgs, deps = [], []
                for i in range(case["n"]):
                    random.seed(case["seed"] + i)
                    s = ds[i]
                    imgs.append(s["image"].numpy())
                    deps.append(s["depth"].numpy())
                out[f"{name}/image"] = np.stack(imgs).astype(np.float32)
                out[f"{name}/depth"] = np.stack(deps).astype(np.float32)
                print(name, out[f"{name}/image"].shape, out[f"{name}/depth"].shape)
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "augment.npz"), **out)


if __name__ == "__main__":
    main()
