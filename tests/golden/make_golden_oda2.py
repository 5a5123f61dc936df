"""Golden fixtures for the ODA2 ordered-swin2 family, generated from the
reference itself.  Run in the build container (the reference never travels):

    python tests/golden/make_golden_oda2.py [--ref /root/reference]

Same conventions as make_golden.py (PCG64 inputs, dropout p=0, BatchNorm in training mode, L = sum(out * dy) with seeded dy), plus:

  * weights come from oracle.weights.rng_fill (seeded full-rank Gaussians; "fillmode" =
    "rng" in each file), not the closed-form sinusoid;
  * timm's DropPath is stubbed to identity (stochastic depth off for parity runs);
  * the ODA2 wrapper hard-codes a Swin-L/B encoder loaded from a checkpoint file
    (model/ODA2/oda2_red_order_swin2.py:30-45).  For the end-to-end fixture the harness
    swaps the SwinTransformer symbol the wrapper module imported for a factory that
    builds the reference's own class at a small width (embed 32, depths 2/2/2/2) and
    makes init_weights a no-op -- the model's forward (resize to 448x672, encoder,
    decoder, x max_depth) runs unchanged;
  * the depth-ordering indices that the reducer head derives from each stage's logit
    (oda2_red_order_swin2_decoder.py:247-253, a floor: discontinuous) are recorded as
    "idx/<k>" so a checker can tell a boundary flip from a real mismatch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import make_golden  # noqa: E402
from make_golden import install_stubs, run_and_save  # noqa: E402
from oracle.weights import rng_fill  # noqa: E402


def prep(model: nn.Module, seed: int, scale: float):
    """make_golden.prep with oracle.weights.rng_fill (full-rank weights) instead of the
    rank-2 closed-form sinusoid: ODA2's stacks of BatchNorm / LayerNorm over those
    amplify fp32 round-off to ~5e-3 (measured), which no 1e-4 parity bar survives."""
    make_golden.prep(model, 0.0, scale)
    rng_fill(model.state_dict(), seed=seed, scale=scale)
    model.__dict__["_fill"] = (float(seed), scale)
    return model


_orig_run_and_save = run_and_save


def run_and_save(name, *a, **kw):  # noqa: F811  (records the fill mode next to the fill)
    _orig_run_and_save(name, *a, **kw)
    path = os.path.join(HERE, f"{name}.npz")
    d = dict(np.load(path))
    d["fillmode"] = np.array("rng")
    np.savez_compressed(path, **d)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    install_stubs()
    sys.path.insert(0, args.ref)
    torch.manual_seed(0)
    torch.set_num_threads(8)
    meta_path = os.path.join(HERE, "meta.json")
    with open(meta_path) as f:
        meta = json.load(f)

    import model.ODA2.oda2_red_order_swin2 as wrapper_mod
    from model.ODA2.oda2_swin_transformer import SwinTransformer, SwinTransformerStage, PatchMerging
    from model.ODA2.oda2_red_order_swin2_decoder import PreNormOrderedSwinSA, OrderedSwinRegHead
    from model.ODA2.oda2_red_order_reg_decoder import PreNormDWConvFF
    from model.ODA2.oda2_red_order_swin2 import ODA2OrderedSwin2RegModel

    # 1. one Swin stage with replicate padding (oda2_swin_transformer.py:12,254-258,325-327):
    #    9x13 pads to 14x14 for the windows and both sides for the 2x2 merge; 10x12 pads to 14x14
    for (H, W) in [(9, 13), (10, 12)]:
        st = prep(SwinTransformerStage(dim=64, depth=2, num_heads=2, window_size=7, downsample=PatchMerging),
                  seed=11, scale=0.08)
        run_and_save(f"oda2_swin_stage_{H}x{W}", st, {"x": ((2, H * W, 64), 61)},
                     lambda m, i, H=H, W=W: (lambda r: (r[0], r[3]))(m(i["x"], H, W)), ["x_out", "x_down"], seed=61)

    # 2. backbone at 244x374.  The patch embedding's replicate pad (oda2_swin_transformer.py:487-491)
    #    passes a 6-tuple to F.pad on an NCHW tensor, so it pads H (by the W remainder) and C (by
    #    the H remainder): only H % 4 == 0 runs at all, and then H grows by (4 - W % 4) % 4
    #    replicated rows while the stride-4 conv floors W: 244x374 -> 246x374 -> 61x93 tokens.
    #    Stages 61x93, 31x47, 16x24, 8x12: every window map pads, every merge sees matching
    #    parity (the reference's swapped merge pad, :326-327, fails otherwise) and every stage
    #    has >= 2 windows per side (its shift-mask .view, :430, fails on a single window row)
    sw = prep(SwinTransformer(embed_dim=32, depths=(2, 2, 2, 2), num_heads=(1, 2, 4, 8), window_size=7,
                              path_drop_prob=0.0), seed=12, scale=0.05)
    run_and_save("oda2_swin_backbone", sw, {"img": ((2, 3, 244, 374), 62)}, lambda m, i: m(i["img"]),
                 ["o0", "o1", "o2", "o3"], seed=62)

    # 3. ordered window self-attention with the depth-index bias (window 8, shift 0 and 4)
    for shift in (0, 4):
        sa = prep(PreNormOrderedSwinSA(64, 4, num_emb=16, window_size=8, shift_size=shift), seed=13, scale=0.05)
        idx = torch.from_numpy(np.random.Generator(np.random.PCG64(63)).integers(0, 16, (2, 16, 24)))
        run_and_save(f"oda2_ordered_sa_shift{shift}", sa, {"x": ((2, 16, 24, 64), 63)},
                     lambda m, i, idx=idx: m(i["x"], idx), ["y", "attn"], seed=63 + shift)

    # 4. pre-norm GLU + depthwise 5x5 (replicate) + BN + GELU feed-forward
    ff = prep(PreNormDWConvFF(32, feedforward_dims=64), seed=14, scale=0.05)
    run_and_save("oda2_dwconv_ff", ff, {"x": ((2, 10, 12, 32), 64)}, lambda m, i: m(i["x"]), ["y"], seed=64)

    # 5. the reducer head alone (3 ordered blocks, conv heads, sigmoid, index feedback)
    hd = prep(OrderedSwinRegHead(64, 4, 2, num_emb=16, window_size=8), seed=15, scale=0.05)
    store_idx = {}

    def head_fwd(m, i):
        orig = m._logit_to_indices
        calls = []

        def rec(out):
            r = orig(out)
            calls.append(r)
            return r
        m._logit_to_indices = rec
        outs, attn = m(i["x"])
        m._logit_to_indices = orig
        store_idx["head"] = [c.numpy() for c in calls]
        return tuple(outs) + tuple(attn)

    run_and_save("oda2_reg_head", hd, {"x": ((2, 16, 24, 64), 65)}, head_fwd,
                 ["out0", "out1", "out2"] + [f"attn{k}" for k in range(4)], seed=65)
    _append_idx("oda2_reg_head", store_idx["head"])

    # 6. end-to-end wrapper at NYU 480x640 (resized to 448x672 inside) with a narrow encoder
    def small_swin(embed_dim, num_heads, **kw):
        kw.update(depths=(2, 2, 2, 2), path_drop_prob=0.0, use_checkpoint=kw.get("use_checkpoint", False))
        m = SwinTransformer(embed_dim=32, num_heads=(1, 2, 4, 8), **kw)
        m.init_weights = lambda pretrained=None: None
        return m

    real = wrapper_mod.SwinTransformer
    wrapper_mod.SwinTransformer = small_swin
    try:
        for neck in ("red", "red33"):
            net = ODA2OrderedSwin2RegModel(dec_dim=64, min_depth=1e-3, max_depth=10.0, num_heads=4, num_repeats=2,
                                           num_emb=16, window_size=8, encoder_type="large", neck_type=neck)
            prep(net, seed=16, scale=0.05)
            calls = []
            orig = net.decoder.reducer._logit_to_indices

            def rec(out, orig=orig, calls=calls):
                r = orig(out)
                calls.append(r)
                return r
            net.decoder.reducer._logit_to_indices = rec

            def fwd(m, i):
                calls.clear()
                out, outs, attn = m(i["img"])
                return (out,) + tuple(outs[:-1])

            name = f"oda2_model_{neck}"
            run_and_save(name, net, {"img": ((1, 3, 480, 640), 66)}, fwd, ["depth", "out0", "out1"],
                         summary=True, seed=66)
            _append_idx(name, [c.numpy() for c in calls])
            meta[name] = {"dec_dim": 64, "num_heads": 4, "num_repeats": 2, "num_emb": 16, "window_size": 8,
                          "neck_type": neck, "max_depth": 10.0, "encoder": {"embed_dim": 32, "depths": [2, 2, 2, 2],
                                                                             "num_heads": [1, 2, 4, 8]},
                          "fill_seed": 16, "fill_scale": 0.05}
    finally:
        wrapper_mod.SwinTransformer = real

    meta["oda2_generator"] = "tests/golden/make_golden_oda2.py"
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1)


def _append_idx(name, arrays):
    path = os.path.join(HERE, f"{name}.npz")
    d = dict(np.load(path))
    for k, a in enumerate(arrays):
        d[f"idx/{k}"] = a.astype(np.int16)
    np.savez_compressed(path, **d)


if __name__ == "__main__":
    main()
