"""EfficientNet-B5 (`tf_efficientnet_b5_ap`) on libmdemi kernels, NHWC inside.

The reference does not contain this network: AdaBins and Depthformer-v8 fetch
it with ``torch.hub.load('rwightman/gen-efficientnet-pytorch',
'tf_efficientnet_b5_ap', pretrained=True)`` (unet_adaptive_bins.py:129,
depthformer_v8.py:89) and then walk ``backend._modules`` (conv_stem, bn1,
act1, blocks[0..6], conv_head, bn2, act2; unet_adaptive_bins.py:65-73,
depthformer_v8.py:15-24).  This module restates that published architecture
(gen-efficientnet @ master, commit unpinned by the reference) with the same
module names, so its state_dict keys are the hub model's:

  * channel multiplier 1.6, depth multiplier 2.2 (ceil), TF 'same' padding
    (asymmetric for stride 2), BatchNorm eps 1e-3, swish;
  * stages ds_r1_k3_s1_e1_c16, ir_r2_k3_s2_e6_c24, ir_r2_k5_s2_e6_c40,
    ir_r3_k3_s2_e6_c80, ir_r3_k5_s1_e6_c112, ir_r4_k5_s2_e6_c192,
    ir_r1_k3_s1_e6_c320, all with SqueezeExcite 0.25 of the block input;
  * stem 48, stage widths 24/40/64/128/176/304/512, head 2048.

No pretrained weights exist offline: ``tf_efficientnet_b5_ap()`` is randomly
initialised.  Parity of this encoder is unpinned.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import _lib as L
from .. import functional as mf
from .NewCRFs.uper_crf_head import bn_forward

BN_EPS_TF = 1e-3  # gen-efficientnet BN_EPS_TF_DEFAULT (tf_* models); momentum stays nn's 0.1


def make_divisible(v, divisor=8, min_value=None):
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def round_channels(channels, multiplier=1.0, divisor=8):
    return make_divisible(channels * multiplier, divisor) if multiplier else channels


class Swish(nn.Module):
    """Placeholder for the activation that follows a BatchNormAct2d (fused into it)."""

    def forward(self, x):
        return x


class BatchNormAct2d(nn.BatchNorm2d):
    """BatchNorm2d (TF eps/momentum) with the following swish fused into the same sweep."""

    def __init__(self, num_features, act=True):
        super().__init__(num_features, eps=BN_EPS_TF)
        self.fused_act = L.ACT_SILU if act else L.ACT_NONE

    def forward(self, x):
        return bn_forward(self, x, self.fused_act)


class Conv2dSame(nn.Conv2d):
    """nn.Conv2d with TF 'same' padding on NHWC; depthwise when groups == channels.  The stem
    (3 input channels) takes the NCHW image and zero-pads its channels to 4."""

    def __init__(self, in_chs, out_chs, k, stride=1, groups=1):
        super().__init__(in_chs, out_chs, k, stride=stride, padding=0, groups=groups, bias=False)

    def forward_skip(self, x):
        """(conv(x), x) of a 1x1 conv whose input is also the block's residual (mf.conv2d_nhwc_skip)."""
        return mf.conv2d_nhwc_skip(x, self.weight)

    def forward(self, x):
        k, s = self.kernel_size[0], self.stride[0]
        if self.groups > 1:
            return mf.dwconv_nhwc(x, self.weight, stride=s, same=True)
        if self.in_channels == 3 and x.dim() == 4 and x.shape[1] == 3:  # conv_stem on the NCHW image
            x = mf.nchw_to_nhwc_pad(x, 4)
            w = torch.nn.functional.pad(self.weight, (0, 0, 0, 0, 0, 1))
        else:
            w = self.weight
        h, wd = x.shape[1], x.shape[2]
        oh, pt = mf.same_pad(h, k, s)
        ow, pl = mf.same_pad(wd, k, s)
        if k == 1 and s == 1:
            return mf.conv2d_nhwc(x, w, None, stride=1, pad=0)
        if pt != pl:
            raise NotImplementedError("asymmetric top/left padding")
        return mf.conv2d_nhwc(x, w, None, stride=s, pad=pt, out_hw=(oh, ow))


class SqueezeExcite(nn.Module):
    def __init__(self, in_chs, reduced_base_chs, se_ratio=0.25):
        super().__init__()
        reduced = make_divisible(reduced_base_chs * se_ratio, 1)
        self.conv_reduce = nn.Conv2d(in_chs, reduced, 1, bias=True)
        self.act1 = Swish()
        self.conv_expand = nn.Conv2d(reduced, in_chs, 1, bias=True)

    def forward(self, x):
        r, c = self.conv_reduce.weight.shape[:2]
        return mf.squeeze_excite(x, self.conv_reduce.weight.view(r, c), self.conv_reduce.bias,
                                 self.conv_expand.weight.view(c, r), self.conv_expand.bias)


def _residual(x, shortcut):
    # the block output feeds the next block's conv_pw (a bf16 GEMM under bf16 storage)
    return mf.add(x, shortcut, out_b16=True)


class DepthwiseSeparableConv(nn.Module):
    """ds block: conv_dw -> bn1+swish -> se -> conv_pw -> bn2 (+ skip)."""

    def __init__(self, in_chs, out_chs, k, stride):
        super().__init__()
        self.has_residual = stride == 1 and in_chs == out_chs
        self.conv_dw = Conv2dSame(in_chs, in_chs, k, stride=stride, groups=in_chs)
        self.bn1 = BatchNormAct2d(in_chs)
        self.bn1._mdemi_pool = True  # its output feeds the SE: the BN sweep also pools it
        self.act1 = Swish()
        self.se = SqueezeExcite(in_chs, in_chs)
        self.conv_pw = Conv2dSame(in_chs, out_chs, 1)
        self.bn2 = BatchNormAct2d(out_chs, act=False)
        self.bn2._mdemi_out_b16 = not self.has_residual  # the block output feeds the next conv_pw
        self.act2 = nn.Identity()

    def forward(self, x):
        y = self.bn2(self.conv_pw(self.se(self.bn1(self.conv_dw(x)))))
        return _residual(y, x) if self.has_residual else y


class InvertedResidual(nn.Module):
    """ir block: conv_pw -> bn1+swish -> conv_dw -> bn2+swish -> se -> conv_pwl -> bn3 (+ skip)."""

    def __init__(self, in_chs, out_chs, k, stride, exp_ratio):
        super().__init__()
        mid = make_divisible(in_chs * exp_ratio)
        self.has_residual = in_chs == out_chs and stride == 1
        self.conv_pw = Conv2dSame(in_chs, mid, 1)
        self.bn1 = BatchNormAct2d(mid)
        self.act1 = Swish()
        self.conv_dw = Conv2dSame(mid, mid, k, stride=stride, groups=mid)
        self.bn2 = BatchNormAct2d(mid)
        self.bn2._mdemi_pool = True  # its output feeds the SE: the BN sweep also pools it
        self.act2 = Swish()
        self.se = SqueezeExcite(mid, in_chs)
        self.conv_pwl = Conv2dSame(mid, out_chs, 1)
        self.bn3 = BatchNormAct2d(out_chs, act=False)
        self.bn3._mdemi_out_b16 = not self.has_residual  # the block output feeds the next conv_pw

    def forward(self, x):
        if self.has_residual:  # x's two gradients meet in conv_pw's input-gradient epilogue
            y, x = self.conv_pw.forward_skip(x)
        else:
            y = self.conv_pw(x)
        y = self.bn2(self.conv_dw(self.bn1(y)))
        y = self.bn3(self.conv_pwl(self.se(y)))
        return _residual(y, x) if self.has_residual else y


# (block type, repeats, kernel, stride, expansion, channels) — EfficientNet-B0 arch, SE 0.25 everywhere
_ARCH = [("ds", 1, 3, 1, 1, 16), ("ir", 2, 3, 2, 6, 24), ("ir", 2, 5, 2, 6, 40), ("ir", 3, 3, 2, 6, 80),
         ("ir", 3, 5, 1, 6, 112), ("ir", 4, 5, 2, 6, 192), ("ir", 1, 3, 1, 6, 320)]


class GenEfficientNet(nn.Module):
    def __init__(self, channel_multiplier=1.6, depth_multiplier=2.2, num_features=1280, stem_size=32,
                 num_classes=1000):
        super().__init__()
        stem = round_channels(stem_size, channel_multiplier)
        self.conv_stem = Conv2dSame(3, stem, 3, stride=2)
        self.bn1 = BatchNormAct2d(stem)
        self.act1 = Swish()
        in_chs = stem
        stages = []
        for bt, r, k, s, e, c in _ARCH:
            out_chs = round_channels(c, channel_multiplier)
            reps = int(math.ceil(r * depth_multiplier))
            blocks = []
            for i in range(reps):
                stride = s if i == 0 else 1
                if bt == "ds":
                    blocks.append(DepthwiseSeparableConv(in_chs, out_chs, k, stride))
                else:
                    blocks.append(InvertedResidual(in_chs, out_chs, k, stride, e))
                in_chs = out_chs
            stages.append(nn.Sequential(*blocks))
        self.blocks = nn.Sequential(*stages)
        self.num_features = round_channels(num_features, channel_multiplier)
        self.conv_head = Conv2dSame(in_chs, self.num_features, 1)
        self.bn2 = BatchNormAct2d(self.num_features)
        self.act2 = Swish()
        self.global_pool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Linear(self.num_features, num_classes)
        for m in self.modules():  # gen-efficientnet _initialize_weight_goog
            if isinstance(m, nn.Conv2d):
                fan_out = m.kernel_size[0] * m.kernel_size[1] * m.out_channels // m.groups
                m.weight.data.normal_(0, math.sqrt(2.0 / fan_out))
                if m.bias is not None:
                    m.bias.data.zero_()
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1.0)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                r = 1.0 / math.sqrt(m.weight.size(0))
                m.weight.data.uniform_(-r, r)
                m.bias.data.zero_()


def tf_efficientnet_b5_ap(pretrained=False, **kwargs):
    """The hub entry point the reference calls; weights cannot be downloaded here."""
    if pretrained:
        print("tf_efficientnet_b5_ap: pretrained weights are not available offline; random init")
    return GenEfficientNet(channel_multiplier=1.6, depth_multiplier=2.2, **kwargs)


def walk_features(backend, x, last):
    """The reference's encoder walk (unet_adaptive_bins.py:65-73 / depthformer_v8.py:15-24):
    features[0] is the image, then one entry per backend module with 'blocks' expanded per
    stage.  Stops after feature index `last`: later entries are never consumed by the decoders
    (AdaBins reads up to [11], Depthformer-v8 up to [10])."""
    features = [x]
    for k, v in backend._modules.items():
        if len(features) > last:
            break
        if k == "blocks":
            for _, vi in v._modules.items():
                if len(features) > last:
                    break
                features.append(vi(features[-1]))
        else:
            features.append(v(features[-1]))
    return features
