"""PSP head (PPM + bottleneck) on libmdemi kernels; mirrors
model/NewCRFs/uper_crf_head.py's PPM / BaseDecodeHead / PSP and mmcv's
ConvModule (conv -> norm -> ReLU, attribute names conv/bn/gn/activate,
bias only without a norm) so the state_dict keys match the reference."""
import torch
import torch.nn as nn

from ... import _lib as L
from ... import functional as mf


class ConvModule(nn.Module):
    """mmcv.cnn.ConvModule as used by uper_crf_head.py (norm BN or GN, act ReLU)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, conv_cfg=None, norm_cfg=None,
                 act_cfg=dict(type="ReLU"), **kwargs):
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
                raise ValueError(f"unsupported norm {t}")
        if act_cfg is not None and act_cfg.get("type") != "ReLU":
            raise ValueError("ConvModule: only ReLU is used by the reference")
        self.activate = nn.ReLU(inplace=True) if act_cfg is not None else None

    def forward(self, x):
        k = self.conv.kernel_size[0]
        y = mf.conv2d_nhwc(x, self.conv.weight, self.conv.bias, stride=self.conv.stride[0], pad=self.conv.padding[0])
        act = L.ACT_RELU if self.activate is not None else L.ACT_NONE
        if self.norm_name == "bn":
            return bn_forward(self.bn, y, act)
        if self.norm_name == "gn":
            return mf.group_norm_nhwc(y, self.gn.weight, self.gn.bias, self.gn.num_groups, self.gn.eps, act)
        if act != L.ACT_NONE:
            raise NotImplementedError("ConvModule without norm but with activation")
        del k
        return y


def bn_forward(bn: nn.BatchNorm2d, x, act=L.ACT_NONE):
    """nn.BatchNorm2d semantics on an NHWC map: batch statistics + running-stat
    update in training, running statistics in eval."""
    if bn.training or not bn.track_running_stats:
        if bn.track_running_stats and bn.momentum is not None:  # statistics + running update, one call
            # _mdemi_out_b16 (set by the model where the BN's output feeds a conv): under bf16
            # storage the same sweep writes the output's bf16 copy for that GEMM
            # _mdemi_pool (set where the output feeds a SqueezeExcite): the sweep also pools it
            y, _, _ = mf.batch_norm_nhwc(x, bn.weight, bn.bias, bn.eps, act,
                                         running=(bn.running_mean, bn.running_var, bn.num_batches_tracked,
                                                  bn.momentum), out_b16=getattr(bn, "_mdemi_out_b16", False),
                                         pool=getattr(bn, "_mdemi_pool", False))
            return y
        y, mean, rstd = mf.batch_norm_nhwc(x, bn.weight, bn.bias, bn.eps, act)
        if bn.track_running_stats:  # cumulative average (momentum None): needs the count on the host
            with torch.no_grad():
                n = x.numel() // x.shape[-1]
                bn.num_batches_tracked.add_(1)
                m = 1.0 / float(bn.num_batches_tracked)
                L.call("mdemi_bn_running_update", mean.data_ptr(), rstd.data_ptr(), bn.running_mean.data_ptr(),
                       bn.running_var.data_ptr(), None, x.shape[-1], n, float(bn.eps), float(m), L.stream())
        return y
    return mf.batch_norm_eval_nhwc(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, act)


class AdaptiveAvgPool2d(nn.AdaptiveAvgPool2d):
    def forward(self, x):
        return mf.adaptive_avg_pool_nhwc(x, self.output_size)


class PPM(nn.ModuleList):
    """uper_crf_head.py:9-58 — note the reference's `norm_cfg` overwrite at
    pool_scale==1 (:35) leaves GroupNorm(256) on all four branches."""

    def __init__(self, pool_scales, in_channels, channels, conv_cfg, norm_cfg, act_cfg, align_corners):
        super().__init__()
        self.pool_scales = pool_scales
        self.align_corners = align_corners
        self.in_channels = in_channels
        self.channels = channels
        self.conv_cfg = conv_cfg
        self.norm_cfg = norm_cfg
        self.act_cfg = act_cfg
        for pool_scale in pool_scales:
            if pool_scale == 1:
                norm_cfg = dict(type="GN", requires_grad=True, num_groups=256)
            self.append(nn.Sequential(AdaptiveAvgPool2d(pool_scale),
                                      ConvModule(self.in_channels, self.channels, 1, conv_cfg=self.conv_cfg,
                                                 norm_cfg=norm_cfg, act_cfg=self.act_cfg)))

    def forward(self, x):
        H, W = x.shape[1], x.shape[2]
        return [mf.interpolate_bilinear(ppm(x), size=(H, W), align_corners=self.align_corners) for ppm in self]


class BaseDecodeHead(nn.Module):
    """uper_crf_head.py:60-200 (only what PSP uses)."""

    def __init__(self, in_channels, channels, *, num_classes, dropout_ratio=0.1, conv_cfg=None, norm_cfg=None,
                 act_cfg=dict(type="ReLU"), in_index=-1, input_transform=None, loss_decode=None, ignore_index=255,
                 sampler=None, align_corners=False):
        super().__init__()
        if input_transform not in (None, "multiple_select"):
            raise NotImplementedError(f"input_transform={input_transform}")
        self.input_transform = input_transform
        self.in_index = in_index
        self.in_channels = in_channels
        self.channels = channels
        self.num_classes = num_classes
        self.dropout_ratio = dropout_ratio
        self.conv_cfg = conv_cfg
        self.norm_cfg = norm_cfg
        self.act_cfg = act_cfg
        self.ignore_index = ignore_index
        self.align_corners = align_corners
        if dropout_ratio > 0:
            raise NotImplementedError("PSP is built with dropout_ratio=0.0 by NewCRFDepth")
        self.dropout = None
        self.fp16_enabled = False

    def init_weights(self):
        pass

    def _transform_inputs(self, inputs):
        if self.input_transform == "multiple_select":
            return [inputs[i] for i in self.in_index]
        return inputs[self.in_index]


class PSP(BaseDecodeHead):
    """uper_crf_head.py:318-364; inputs/outputs NHWC."""

    def __init__(self, pool_scales=(1, 2, 3, 6), **kwargs):
        super().__init__(input_transform="multiple_select", **kwargs)
        self.psp_modules = PPM(pool_scales, self.in_channels[-1], self.channels, conv_cfg=self.conv_cfg,
                               norm_cfg=self.norm_cfg, act_cfg=self.act_cfg, align_corners=self.align_corners)
        self.bottleneck = ConvModule(self.in_channels[-1] + len(pool_scales) * self.channels, self.channels, 3,
                                     padding=1, conv_cfg=self.conv_cfg, norm_cfg=self.norm_cfg, act_cfg=self.act_cfg)

    def psp_forward(self, inputs):
        x = inputs[-1]
        cat = mf.concat_channels([x] + self.psp_modules(x))
        return self.bottleneck(cat)

    def forward(self, inputs):
        return self.psp_forward(self._transform_inputs(inputs))
