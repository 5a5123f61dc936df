"""CPU restatement of EfficientNet-B5 (`tf_efficientnet_b5_ap`, rwightman/gen-
efficientnet-pytorch, the encoder AdaBins and Depthformer-v8 fetch with
torch.hub: unet_adaptive_bins.py:129, depthformer_v8.py:89).  TEST
INFRASTRUCTURE ONLY — see oracle/__init__.py.

PARITY UNPINNED: the network is third-party, not in /root/reference, and
cannot be fetched offline; this restates its published architecture (TF
'same' padding via Conv2dSame, BN eps 1e-3, swish, SqueezeExcite 0.25 of the
block input, channel x1.6 / depth x2.2) in plain torch ops on the state_dict
keys of the hub model.  The reference pins only the interface: channel counts
(unet_adaptive_bins.py:34-37, depthformer_v8.py:37), feature indices
(unet_adaptive_bins.py:44-45, depthformer_v8.py:58) and the walk itself
(unet_adaptive_bins.py:65-73).
"""
import math

import torch
import torch.nn.functional as F

from . import bf16emu as E
from . import bnmode

BN_EPS = 1e-3
# (block type, repeats, kernel, stride, expansion, channels) of EfficientNet-B0, scaled below
ARCH = [("ds", 1, 3, 1, 1, 16), ("ir", 2, 3, 2, 6, 24), ("ir", 2, 5, 2, 6, 40), ("ir", 3, 3, 2, 6, 80),
        ("ir", 3, 5, 1, 6, 112), ("ir", 4, 5, 2, 6, 192), ("ir", 1, 3, 1, 6, 320)]


def conv_same(x, w, stride=1, groups=1, b=None):
    """gen-efficientnet Conv2dSame / static 'same' padding: output ceil(in/stride)."""
    k = w.shape[-1]
    ih, iw = x.shape[-2:]
    ph = max((math.ceil(ih / stride) - 1) * stride + k - ih, 0)
    pw = max((math.ceil(iw / stride) - 1) * stride + k - iw, 0)
    if ph or pw:
        x = F.pad(x, [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2])
    return E.conv2d(x, w, b, stride=stride, groups=groups)


def bn(P, pre, x):
    return bnmode.batch_norm(P, pre, x, BN_EPS)


def se(P, pre, x):
    s = x.mean((2, 3), keepdim=True)
    s = F.silu(F.conv2d(s, P[pre + "conv_reduce.weight"], P[pre + "conv_reduce.bias"]))
    s = F.conv2d(s, P[pre + "conv_expand.weight"], P[pre + "conv_expand.bias"])
    return x * torch.sigmoid(s)


def ds_block(P, pre, x, stride, residual):
    w = P[pre + "conv_dw.weight"]
    y = F.silu(bn(P, pre + "bn1.", conv_same(x, w, stride, groups=w.shape[0])))
    y = se(P, pre + "se.", y)
    y = bn(P, pre + "bn2.", E.conv2d(y, P[pre + "conv_pw.weight"]))
    return y + x if residual else y


def ir_block(P, pre, x, stride, residual):
    y = F.silu(bn(P, pre + "bn1.", E.conv2d(x, P[pre + "conv_pw.weight"])))
    w = P[pre + "conv_dw.weight"]
    y = F.silu(bn(P, pre + "bn2.", conv_same(y, w, stride, groups=w.shape[0])))
    y = se(P, pre + "se.", y)
    y = bn(P, pre + "bn3.", E.conv2d(y, P[pre + "conv_pwl.weight"]))
    return y + x if residual else y


def features(P, pre, x, last=11, depth_multiplier=2.2):
    """The encoder walk: [x, conv_stem, bn1, act1, stage 0..6, conv_head, act2][:last + 1]
    (unet_adaptive_bins.py:65-73).  bn1 output is returned post-swish at index 2 and 3."""
    feats = [x]
    y = conv_same(x, P[pre + "conv_stem.weight"], 2)
    feats.append(y)
    y = F.silu(bn(P, pre + "bn1.", y))
    feats += [y, y]
    for si, (bt, r, k, s, e, c) in enumerate(ARCH):
        reps = int(math.ceil(r * depth_multiplier))
        for i in range(reps):
            bp = f"{pre}blocks.{si}.{i}."
            stride = s if i == 0 else 1
            cin = y.shape[1]
            cout = P[bp + ("conv_pw.weight" if bt == "ds" else "conv_pwl.weight")].shape[0]
            res = stride == 1 and cin == cout
            y = ds_block(P, bp, y, stride, res) if bt == "ds" else ir_block(P, bp, y, stride, res)
        feats.append(y)
        if len(feats) > last:
            return feats
    if pre + "conv_head.weight" in P:
        feats.append(E.conv2d(y, P[pre + "conv_head.weight"]))
    return feats[:last + 1]
