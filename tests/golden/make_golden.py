"""Generate golden fixtures from the reference implementation itself.

Run in the build container (the reference lives at /root/reference and never
travels to the GPU box):

    python tests/golden/make_golden.py [--ref /root/reference]

What it does
  * imports the reference's model modules as-is (AdaBins, Depthformer v8) or
    with harness-only stubs (NewCRFs needs timm.models.layers, mmcv.cnn and
    torchvision, none of which are installed; the stubs restate only what the
    reference uses: DropPath -> identity (parity runs have stochastic depth
    off), to_2tuple, trunc_normal_, and mmcv's ConvModule conv->norm->act with
    its `conv`/`bn`/`gn`/`activate` attribute names and bias='auto').
  * fills every floating state_dict entry with the closed-form sequence of
    oracle/weights.py (so the GPU box regenerates identical weights from the
    formula, with no weight files), draws inputs from numpy PCG64(seed),
    switches every Dropout (and nn.MultiheadAttention's dropout) to p=0, keeps BatchNorm in training mode.
  * runs forward, then backward of L = sum(out * dy) with a seeded dy, and
    stores inputs, outputs and gradients in small .npz files.

Stored names: "in/<x>", "out/<y>", "dy/<y>", "grad/<x or param>", and for the
end-to-end models "gsum/<param>" = [sum, sum of squares] of the gradient.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle.weights import closed_form_fill, rng_array  # noqa: E402


# ---------------------------------------------------------------------------
# harness-only stubs for third-party packages absent from this image
# ---------------------------------------------------------------------------
def install_stubs():
    timm = types.ModuleType("timm")
    timm_models = types.ModuleType("timm.models")
    timm_layers = types.ModuleType("timm.models.layers")

    class DropPath(nn.Module):  # stochastic depth is switched off for parity runs
        def __init__(self, drop_prob=None):
            super().__init__()
            self.drop_prob = drop_prob

        def forward(self, x):
            return x

    def to_2tuple(x):
        return tuple(x) if isinstance(x, (list, tuple)) else (x, x)

    def trunc_normal_(tensor, mean=0.0, std=1.0, a=-2.0, b=2.0):
        return nn.init.trunc_normal_(tensor, mean, std, a, b)

    timm_layers.DropPath = DropPath
    timm_layers.to_2tuple = to_2tuple
    timm_layers.trunc_normal_ = trunc_normal_
    timm.models = timm_models
    timm_models.layers = timm_layers
    sys.modules.update({"timm": timm, "timm.models": timm_models, "timm.models.layers": timm_layers})

    mmcv = types.ModuleType("mmcv")
    mmcv_cnn = types.ModuleType("mmcv.cnn")

    class ConvModule(nn.Module):
        """conv -> norm -> act with mmcv's attribute names; bias='auto' = no bias when normed."""

        def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, conv_cfg=None,
                     norm_cfg=None, act_cfg=dict(type="ReLU"), **kw):
            super().__init__()
            with_norm = norm_cfg is not None
            self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                                  bias=not with_norm)
            self.norm_name = None
            if with_norm:
                t = norm_cfg["type"]
                if t == "BN":
                    self.norm_name = "bn"
                    self.add_module("bn", nn.BatchNorm2d(out_channels))
                elif t == "GN":
                    self.norm_name = "gn"
                    self.add_module("gn", nn.GroupNorm(norm_cfg["num_groups"], out_channels))
                else:
                    raise ValueError(t)
            self.activate = nn.ReLU(inplace=True) if act_cfg is not None else None

        def forward(self, x):
            x = self.conv(x)
            if self.norm_name:
                x = getattr(self, self.norm_name)(x)
            if self.activate is not None:
                x = self.activate(x)
            return x

    mmcv_cnn.ConvModule = ConvModule
    mmcv.cnn = mmcv_cnn
    sys.modules.update({"mmcv": mmcv, "mmcv.cnn": mmcv_cnn})
    sys.modules.setdefault("torchvision", types.ModuleType("torchvision"))


def prep(model: nn.Module, seed: float, scale: float):
    closed_form_fill(model.state_dict(), seed=seed, scale=scale)
    model.__dict__["_fill"] = (seed, scale)
    for m in model.modules():
        if isinstance(m, nn.Dropout):
            m.p = 0.0
        if isinstance(m, nn.MultiheadAttention):  # attention dropout is a float attribute, not a module
            m.dropout = 0.0
    model.train()
    return model


BIG = 20_000  # elements; larger arrays are stored as a strided subsample + (sum, sum of squares)


def put(store, key, arr):
    arr = np.asarray(arr)
    if arr.size <= BIG:
        store[key] = arr
    else:
        flat = arr.reshape(-1).astype(np.float64)
        step = int(np.ceil(arr.size / 4_000))
        store["sub/" + key] = flat[::step].astype(arr.dtype)
        store["substep/" + key] = np.array(step)
        store["sum/" + key] = np.array([flat.sum(), (flat * flat).sum()])


def run_and_save(name, model, inputs: dict, fwd, out_names, param_grads=True, summary=False, seed=0):
    """inputs: name -> (shape, seed); arrays come from oracle.weights.rng_array."""
    model.zero_grad(set_to_none=True)
    ins = {k: torch.from_numpy(rng_array(shp, sd)).requires_grad_() for k, (shp, sd) in inputs.items()}
    outs = fwd(model, ins)
    if not isinstance(outs, (tuple, list)):
        outs = (outs,)
    store = {}
    loss = 0.0
    for i, (oname, o) in enumerate(zip(out_names, outs)):
        if oname is None:
            continue
        dseed = seed + 100 + i
        dy = rng_array(tuple(o.shape), seed=dseed)
        put(store, f"out/{oname}", o.detach().numpy())
        store[f"dyseed/{oname}"] = np.array(dseed)
        loss = loss + (o * torch.from_numpy(dy)).sum()
    loss.backward()
    for k, v in ins.items():
        store[f"inshape/{k}"] = np.array(v.shape)
        store[f"inseed/{k}"] = np.array(inputs[k][1])
        if v.grad is not None:
            put(store, f"grad/{k}", v.grad.numpy())
    for pn, p in model.named_parameters():
        if p.grad is None:
            continue
        if summary:
            g = p.grad.double()
            store[f"gsum/{pn}"] = np.array([g.sum().item(), (g * g).sum().item()])
        elif param_grads:
            put(store, f"grad/{pn}", p.grad.numpy())
    spec = [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in model.state_dict().items()]
    store["spec"] = np.array(json.dumps(spec))
    store["fill"] = np.array(model.__dict__["_fill"], dtype=np.float64)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **store)
    print(f"{name}: {len(store)} arrays, {os.path.getsize(path) / 1024:.0f} KiB")


class Const(nn.Module):
    """Stands in for an EfficientNet stage: returns a stored feature map (no params)."""

    def __init__(self, holder, idx):
        super().__init__()
        self.__dict__["_holder"] = holder
        self.idx = idx

    def forward(self, x):
        return self._holder[self.idx]


def fake_effnet(holder):
    """Module tree walked like gen-efficientnet's: conv_stem,bn1,act1,blocks[0..6],conv_head,act2.
    Feature list index k (features[0] is the image) returns holder[k]."""
    m = nn.Module()
    m.conv_stem = Const(holder, 1)
    m.bn1 = Const(holder, 2)
    m.act1 = Const(holder, 3)
    m.blocks = nn.Sequential(*[Const(holder, 4 + i) for i in range(7)])
    m.conv_head = Const(holder, 11)
    m.act2 = Const(holder, 12)
    return m


EFF_CH = {4: 24, 5: 40, 6: 64, 7: 128, 8: 176, 9: 304, 10: 512, 11: 2048, 12: 2048}
EFF_STRIDE = {4: 2, 5: 4, 6: 8, 7: 16, 8: 16, 9: 32, 10: 32, 11: 32, 12: 32}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    install_stubs()
    sys.path.insert(0, args.ref)
    torch.manual_seed(0)
    torch.set_num_threads(8)
    meta = {"generator": "tests/golden/make_golden.py", "torch": torch.__version__}

    from model.NewCRFs.swin_transformer import WindowAttention, BasicLayer, PatchMerging, SwinTransformer
    from model.NewCRFs.newcrf_layers import NewCRF
    from model.NewCRFs.uper_crf_head import PSP
    from model.NewCRFs.NewCRFDepth import NewCRFDepth, DispHead
    from model.Adabins.unet_adaptive_bins import UnetAdaptiveBins
    from model.Adabins.miniViT import mViT
    from model.Depthformer.depthformer_v8 import DepthformerV8
    from utils.depth_utils import tcompute_errors, cal_eval_mask

    # 1. WindowAttention, no mask / with mask (swin_transformer.py:112-144)
    wa = prep(WindowAttention(64, (7, 7), 2), seed=0.1, scale=0.1)
    run_and_save("swin_window_attention", wa, {"x": ((6, 49, 64), 1)}, lambda m, i: m(i["x"]), ["y"], seed=1)
    # mask: -100 where rng_array((3,49,49), 2) > 0.3 else 0 (as BasicLayer builds it, values 0/-100)
    run_and_save("swin_window_attention_mask", wa, {"x": ((6, 49, 64), 1), "mask": ((3, 49, 49), 2)},
                 lambda m, i: m(i["x"], mask=torch.where(i["mask"].detach() > 0.3, -100.0, 0.0)), ["y"], seed=2)

    # 2. BasicLayer (2 blocks W-MSA + SW-MSA, pad to x7, mask, PatchMerging) at 10x12 and 9x13
    for (H, W) in [(10, 12), (9, 13)]:
        bl = prep(BasicLayer(dim=64, depth=2, num_heads=2, window_size=7, downsample=PatchMerging), seed=0.2,
                  scale=0.08)
        run_and_save(f"swin_basic_layer_{H}x{W}", bl, {"x": ((2, H * W, 64), 3)},
                     lambda m, i, H=H, W=W: (lambda r: (r[0], r[3]))(m(i["x"], H, W)), ["x_out", "x_down"], seed=3)

    # 3. Swin backbone (head_dim 32), 2x3x64x96, stochastic depth off
    sw = prep(SwinTransformer(embed_dim=64, depths=[2, 2, 2, 2], num_heads=[2, 4, 8, 16], window_size=7,
                              drop_path_rate=0.0), seed=0.3, scale=0.05)
    run_and_save("swin_backbone", sw, {"img": ((2, 3, 64, 96), 4)}, lambda m, i: m(i["img"]), ["o0", "o1", "o2", "o3"], seed=4)

    # 4. NewCRF layer (proj_x 96->128, proj_v 64->128, 2 CRF blocks, 4 heads)
    crf = prep(NewCRF(input_dim=96, embed_dim=128, window_size=7, v_dim=64, num_heads=4), seed=0.4, scale=0.05)
    run_and_save("newcrf_layer", crf, {"x": ((2, 96, 10, 12), 5), "v": ((2, 64, 10, 12), 6)},
                 lambda m, i: m(i["x"], i["v"]), ["y"], seed=5)

    # 5. PSP head (PPM 1/2/3/6 with the GroupNorm(256) override, bottleneck conv3x3+BN+ReLU)
    psp = prep(PSP(in_channels=[16, 32, 64, 128], in_index=[0, 1, 2, 3], pool_scales=(1, 2, 3, 6), channels=512,
                   dropout_ratio=0.0, num_classes=32, norm_cfg=dict(type="BN", requires_grad=True),
                   align_corners=False), seed=0.5, scale=0.03)
    feats = {f"f{k}": ((2, c, 5 * 2 ** (3 - k), 6 * 2 ** (3 - k)), 7 + k)
             for k, c in enumerate([16, 32, 64, 128])}
    run_and_save("psp_head", psp, feats, lambda m, i: m([i["f0"], i["f1"], i["f2"], i["f3"]]), ["y"], seed=7)

    # 6. DispHead + x4 bilinear (NewCRFDepth.py:151-164,185-188)
    dh = prep(DispHead(input_dim=128), seed=0.6, scale=0.05)
    run_and_save("disp_head", dh, {"x": ((2, 128, 10, 12), 12)}, lambda m, i: m(i["x"], 4), ["y"],
                 seed=12)

    # 7. End-to-end NewCRFDepth('tiny07') at 2x3x64x96 (gradient summaries for parameters)
    nc = NewCRFDepth(version="tiny07", inv_depth=False, max_depth=10.0)
    prep(nc, seed=0.7, scale=0.02)
    run_and_save("newcrfs_tiny07", nc, {"img": ((2, 3, 64, 96), 13)}, lambda m, i: m(i["img"]),
                 ["depth"], summary=True, seed=13)
    meta["newcrfs_tiny07"] = {"version": "tiny07", "max_depth": 10.0, "fill_seed": 0.7, "fill_scale": 0.02}

    # 8. AdaBins non-encoder path with EfficientNet-B5-shaped features (2x3x64x96 image)
    holder = {}
    ada = UnetAdaptiveBins(fake_effnet(holder), n_bins=256, min_val=1e-3, max_val=10.0)
    prep(ada, seed=0.8, scale=0.02)
    AH, AW = 352, 384  # decoder output 176x192 -> 11x12 = 132 patch tokens >= 1 + 128 queries
    fe = {f"f{k}": ((1, EFF_CH[k], AH // EFF_STRIDE[k], AW // EFF_STRIDE[k]), 20 + k) for k in (4, 5, 6, 8, 11)}

    def ada_fwd(m, i):
        holder.clear()
        for k in range(1, 13):
            holder[k] = i.get(f"f{k}", torch.zeros(1))
        return m(torch.zeros(1, 3, AH, AW))

    run_and_save("adabins_head", ada, fe, ada_fwd, ["pred", "bin_edges"], seed=20)
    meta["adabins_head"] = {"img": [AH, AW], "n_bins": 256, "min_val": 1e-3, "max_val": 10.0, "fill_seed": 0.8, "fill_scale": 0.02}

    # 9. mViT standalone (128-channel 176x192 map, 16x16 patches -> 132 tokens)
    mv = prep(mViT(128, n_query_channels=128, patch_size=16, dim_out=256, embedding_dim=128, norm="linear"),
              seed=0.9, scale=0.02)
    run_and_save("mvit", mv, {"x": ((1, 128, 176, 192), 30)}, lambda m, i: m(i["x"]),
                 ["bin_widths", "range_maps"], seed=30)

    # 10. Depthformer v8 (decoder + bin head) with EfficientNet-shaped features
    holder2 = {}
    opt = {"hidden_dim": 64, "num_heads": 4, "num_bins": 32, "num_aux": 16, "img_size": [64, 96],
           "attn_drop_prob": 0.0, "drop_prob": 0.0}
    dfm = DepthformerV8(fake_effnet(holder2), opt, min_depth=1e-3, max_depth=10.0)
    prep(dfm, seed=1.0, scale=0.03)
    fe2 = {f"f{k}": ((2, EFF_CH[k], 64 // EFF_STRIDE[k], 96 // EFF_STRIDE[k]), 40 + k) for k in (4, 5, 6, 8, 10)}

    def dfm_fwd(m, i):
        holder2.clear()
        for k in range(1, 13):
            holder2[k] = i.get(f"f{k}", torch.zeros(1))
        depth, centers, attn = m(torch.zeros(2, 3, 64, 96))
        return (depth, centers) + tuple(attn)

    run_and_save("depthformer_v8", dfm, fe2, dfm_fwd,
                 ["depth", "centers"] + [f"attn{k}" for k in range(8)], seed=40)
    meta["depthformer_v8"] = {"opt": opt, "min_depth": 1e-3, "max_depth": 10.0, "fill_seed": 1.0,
                              "fill_scale": 0.03}

    # 11. depth metrics known answers (utils/depth_utils.py)
    rs = np.random.Generator(np.random.PCG64(50))
    gt = rs.uniform(0.5, 10.0, size=(480, 640)).astype(np.float32)
    pred = (gt * rs.uniform(0.8, 1.25, size=gt.shape)).astype(np.float32)
    store = {"in/gt": gt, "in/pred": pred}
    for name, eo, dt in [("nyu_eigen", {"garg_crop": False, "eigen_crop": True}, "NYU"),
                         ("kitti_garg", {"garg_crop": True, "eigen_crop": False}, "KITTI"),
                         ("kitti_eigen", {"garg_crop": False, "eigen_crop": True}, "KITTI")]:
        mask = cal_eval_mask(eo, gt, dt)
        store[f"mask/{name}"] = mask.astype(np.uint8)
        errs = tcompute_errors(gt[mask], pred[mask])
        for k, v in errs.items():
            store[f"err/{name}/{k}"] = np.array(v, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "depth_metrics.npz"), **store)
    print("depth_metrics written")

    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
