"""Pin the CPU oracle (oracle/) against golden vectors produced by the reference
itself (tests/golden/make_golden.py).  CPU-only; runs in the default suite."""
import os

import numpy as np
import pytest
import torch

from golden_util import GOLDEN, Golden
from oracle import adabins as oab
from oracle import depthformer as odf
from oracle import metrics as omet
from oracle import newcrfs as onc

DT = torch.float32  # the reference's dtype: the restatement should agree to rounding
RT_OUT, RT_GRAD = 2e-5, 2e-4


def _run(g, fwd, out_names, P=None):
    P = P if P is not None else g.params(DT)
    for v in P.values():
        if torch.is_floating_point(v):
            v.requires_grad_(True)
    ins = {n: g.input(n, DT).requires_grad_(True) for n in g.input_names()}
    outs = fwd(P, ins)
    if not isinstance(outs, (tuple, list)):
        outs = (outs,)
    loss = 0
    for name, o in zip(out_names, outs):
        g.check(f"out/{name}", o, RT_OUT, 1e-6)
        loss = loss + (o * g.dy(name, o.shape, DT)).sum()
    loss.backward()
    for n, t in ins.items():
        if g.has(f"grad/{n}"):
            g.check(f"grad/{n}", t.grad, RT_GRAD, 1e-6)
    checked = 0
    for k, v in P.items():
        if g.has(f"grad/{k}"):
            g.check(f"grad/{k}", v.grad, RT_GRAD, 1e-6)
            checked += 1
        elif f"gsum/{k}" in g.d:
            s = g.d[f"gsum/{k}"]
            gv = v.grad.double()
            assert abs(gv.sum().item() - s[0]) <= 1e-3 * np.sqrt(s[1] * gv.numel()) + 1e-6, k
            assert abs((gv * gv).sum().item() - s[1]) <= 1e-3 * s[1] + 1e-12, k
            checked += 1
    return checked


def test_swin_window_attention():
    g = Golden("swin_window_attention")
    _run(g, lambda P, i: onc.window_attention(P, "", i["x"], None, 2, 7), ["y"])


def test_swin_window_attention_mask():
    g = Golden("swin_window_attention_mask")
    _run(g, lambda P, i: onc.window_attention(P, "", i["x"], torch.where(i["mask"].detach() > 0.3, -100.0, 0.0), 2,
                                              7), ["y"])


@pytest.mark.parametrize("hw", [(10, 12), (9, 13)])
def test_swin_basic_layer(hw):
    H, W = hw
    g = Golden(f"swin_basic_layer_{H}x{W}")

    def f(P, i):
        r = onc.basic_layer(P, "", i["x"], H, W, 2, 2, 7, True)
        return r[0], r[3]

    assert _run(g, f, ["x_out", "x_down"]) > 10


def test_swin_backbone():
    g = Golden("swin_backbone")
    _run(g, lambda P, i: onc.swin_transformer(P, "", i["img"], [2, 2, 2, 2], [2, 4, 8, 16], 7),
         ["o0", "o1", "o2", "o3"])


def test_newcrf_layer():
    g = Golden("newcrf_layer")
    _run(g, lambda P, i: onc.newcrf(P, "", i["x"], i["v"], 4), ["y"])


def test_psp_head():
    g = Golden("psp_head")
    _run(g, lambda P, i: onc.psp(P, "", [i["f0"], i["f1"], i["f2"], i["f3"]]), ["y"])


def test_disp_head():
    g = Golden("disp_head")
    _run(g, lambda P, i: onc.disp_head(P, "", i["x"], 4), ["y"])


def test_newcrfs_tiny07_end_to_end():
    g = Golden("newcrfs_tiny07")
    n = _run(g, lambda P, i: onc.newcrf_depth(P, i["img"], "tiny07", max_depth=10.0), ["depth"])
    assert n == sum(1 for k in g.d.keys() if k.startswith("gsum/"))


def _feats(ins, idx):
    feats = [None] * 13
    for k in idx:
        feats[k] = ins[f"f{k}"]
    return feats


def test_adabins_head():
    g = Golden("adabins_head")
    _run(g, lambda P, i: oab.adabins_head(P, _feats(i, (4, 5, 6, 8, 11)), 1e-3, 10.0), ["pred", "bin_edges"])


def test_mvit():
    g = Golden("mvit")
    _run(g, lambda P, i: oab.mvit(P, "", i["x"]), ["bin_widths", "range_maps"])


def test_depthformer_v8():
    g = Golden("depthformer_v8")
    opt = {"hidden_dim": 64, "num_heads": 4, "num_bins": 32, "num_aux": 16}

    def f(P, i):
        feats = [i[f"f{k}"] for k in (4, 5, 6, 8, 10)]
        depth, centers, attn = odf.depthformer_v8(P, feats, opt, 1e-3, 10.0)
        return (depth, centers) + tuple(attn)

    _run(g, f, ["depth", "centers"] + [f"attn{k}" for k in range(8)])


def test_depth_metrics_known_answers():
    d = np.load(os.path.join(GOLDEN, "depth_metrics.npz"))
    gt, pred = d["in/gt"], d["in/pred"]
    for name, eo, dt in [("nyu_eigen", {"garg_crop": False, "eigen_crop": True}, "NYU"),
                         ("kitti_garg", {"garg_crop": True, "eigen_crop": False}, "KITTI"),
                         ("kitti_eigen", {"garg_crop": False, "eigen_crop": True}, "KITTI")]:
        m = omet.cal_eval_mask(eo, gt, dt)
        assert (m == d[f"mask/{name}"].astype(bool)).all()
        errs = omet.compute_errors(gt[m], pred[m])
        for k, v in errs.items():
            assert np.isclose(v, d[f"err/{name}/{k}"], rtol=1e-6, atol=0), (name, k)
