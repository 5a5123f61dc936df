"""Shared helpers for the golden fixtures (tests/golden/*.npz, written by
tests/golden/make_golden.py from the reference itself)."""
import json
import os
from collections import OrderedDict

import numpy as np
import torch

from oracle.newcrfs import relative_position_index
from oracle.weights import closed_form_fill, rng_array

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class Golden:
    def __init__(self, name):
        self.name = name
        self.d = np.load(os.path.join(GOLDEN, name + ".npz"))
        self.spec = json.loads(str(self.d["spec"]))
        self.fill = tuple(float(x) for x in self.d["fill"])

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
