"""Pin the ODA2 CPU oracle (oracle/oda2.py) against golden vectors produced by the reference
itself (tests/golden/make_golden_oda2.py).  CPU-only; runs in the default suite."""
import json
import os
import re

import numpy as np
import pytest
import torch

from golden_util import GOLDEN, Golden
from oracle import oda2 as oo

DT = torch.float32
RT_OUT, RT_GRAD = 2e-5, 2e-4
# Parameters whose gradient is exactly zero in exact arithmetic, so fp32 runs hold only
# round-off there (compared in size, not value):
#  * encoder.norm<i>.bias: every encoder output feeds a (replicate-padded) conv followed by a
#    train-mode BatchNorm (oda2_red_order_swin2_decoder.py:316-343, ConvBN
#    oda2_layer_utils.py:47-50), which removes any per-channel constant;
#  * *.k_proj.bias: adds one constant to every score of a query row, which softmax ignores;
#  * the last ordered block's output-norm bias (reducer.attn_layers.<last>.norm.bias): it
#    reaches the loss only through the last conv head, again a conv + train-mode BatchNorm.
VANISHING = re.compile(r"(^|\.)(encoder\.norm\d\.bias|k_proj\.bias|reducer\.attn_layers\.1\.norm\.bias)$")


def _run(g, fwd, out_names, rt_grad=RT_GRAD):
    P = g.params(DT)
    for v in P.values():
        if torch.is_floating_point(v):
            v.requires_grad_(True)
    ins = {n: g.input(n, DT).requires_grad_(True) for n in g.input_names()}
    outs = fwd(P, ins)
    loss = 0
    for name, o in zip(out_names, outs):
        g.check(f"out/{name}", o, RT_OUT, 1e-6)
        loss = loss + (o * g.dy(name, o.shape, DT)).sum()
    loss.backward()
    for n, t in ins.items():
        if g.has(f"grad/{n}"):
            g.check(f"grad/{n}", t.grad, rt_grad, 1e-6)
    checked = 0
    for k, v in P.items():
        if VANISHING.search(k) and (g.has(f"grad/{k}") or f"gsum/{k}" in g.d):
            ref = float(np.sqrt(g.d[f"gsum/{k}"][1])) if f"gsum/{k}" in g.d else \
                float(np.linalg.norm(g.d.get(f"grad/{k}", g.d.get(f"sub/grad/{k}"))))
            assert v.grad.double().norm().item() <= 10 * ref + 1e-9, k
            checked += 1
        elif g.has(f"grad/{k}"):
            g.check(f"grad/{k}", v.grad, rt_grad, 1e-6)
            checked += 1
        elif f"gsum/{k}" in g.d:
            s = g.d[f"gsum/{k}"]
            gv = v.grad.double()
            assert abs(gv.sum().item() - s[0]) <= 1e-3 * np.sqrt(s[1] * gv.numel()) + 1e-6, k
            assert abs((gv * gv).sum().item() - s[1]) <= 1e-3 * s[1] + 1e-12, k
            checked += 1
    return checked


@pytest.mark.parametrize("hw", [(9, 13), (10, 12)])
def test_oda2_swin_stage_replicate_pad(hw):
    H, W = hw
    g = Golden(f"oda2_swin_stage_{H}x{W}")

    def f(P, i):
        r = oo.stage(P, "", i["x"], H, W, 2, 2, 7, True)
        return r[0], r[3]

    assert _run(g, f, ["x_out", "x_down"]) > 10


def test_oda2_swin_backbone():
    g = Golden("oda2_swin_backbone")
    _run(g, lambda P, i: oo.swin_transformer(P, "", i["img"], (2, 2, 2, 2), (1, 2, 4, 8)), ["o0", "o1", "o2", "o3"])


@pytest.mark.parametrize("shift", [0, 4])
def test_oda2_ordered_sa(shift):
    g = Golden(f"oda2_ordered_sa_shift{shift}")
    idx = torch.from_numpy(np.random.Generator(np.random.PCG64(63)).integers(0, 16, (2, 16, 24)))
    _run(g, lambda P, i: oo.ordered_sa(P, "", i["x"], idx, 4, 8, shift, 16), ["y", "attn"])


def test_oda2_dwconv_ff():
    g = Golden("oda2_dwconv_ff")
    _run(g, lambda P, i: (oo.dwconv_ff(P, "", i["x"]),), ["y"])


def _golden_idx(g):
    return [torch.from_numpy(g.d[f"idx/{k}"].astype(np.int64)) for k in range(len(g.keys("idx/")))]


def test_oda2_reg_head():
    g = Golden("oda2_reg_head")
    want = _golden_idx(g)
    used = []

    def f(P, i):
        outs, attn, u = oo.reg_head(P, "", i["x"], 4, 2, 16, 8)
        used.extend(u)
        return tuple(outs) + tuple(attn)

    _run(g, f, ["out0", "out1", "out2"] + [f"attn{k}" for k in range(4)])
    for a, b in zip(used, want):  # the oracle's own floor() lands on the reference's indices
        assert torch.equal(a, b)


@pytest.mark.parametrize("neck", ["red", "red33"])
def test_oda2_model_end_to_end(neck):
    g = Golden(f"oda2_model_{neck}")
    with open(os.path.join(GOLDEN, "meta.json")) as f:
        meta = json.load(f)[f"oda2_model_{neck}"]
    enc = {"depths": meta["encoder"]["depths"], "num_heads": meta["encoder"]["num_heads"]}
    dec = {"num_heads": meta["num_heads"], "num_repeats": meta["num_repeats"], "num_emb": meta["num_emb"],
           "window_size": meta["window_size"], "neck_type": neck}
    want = _golden_idx(g)
    used = []

    def f(P, i):
        out, outs, attn, u = oo.oda2_model(P, i["img"], enc, dec, meta["max_depth"])
        used.extend(u)
        return (out,) + tuple(outs[:-1])

    n = _run(g, f, ["depth", "out0", "out1"])
    assert n == sum(1 for k in g.d.keys() if k.startswith("gsum/"))
    for a, b in zip(used, want):
        assert (a != b).sum().item() == 0
