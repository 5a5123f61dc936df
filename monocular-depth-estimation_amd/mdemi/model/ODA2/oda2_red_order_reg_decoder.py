"""The feed-forward blocks of model/ODA2/oda2_red_order_reg_decoder.py that the ordered-swin2
decoder imports (PreNormFF, PreNormDWConvFF) on libmdemi kernels, NHWC (B, H, W, C)."""
import math
from typing import Optional

import torch.nn as nn

from ... import _lib as L
from ... import functional as mf
from ..NewCRFs.uper_crf_head import bn_forward
from .oda2_layer_utils import _CONV_PADDING_MODE


class PreNormFF(nn.Module):
    """:11-41 x + drop(lin2(drop(GELU(lin1(LN(x))))))."""

    def __init__(self, in_dims: int, drop_prob: float = 0.0, feedforward_dims: Optional[int] = None,
                 act_layer=nn.GELU):
        super().__init__()
        if feedforward_dims is None:
            feedforward_dims = 4 * in_dims
        self.in_dims = in_dims
        self.norm = nn.LayerNorm(in_dims)
        self.lin1 = nn.Linear(in_dims, feedforward_dims)
        self.lin2 = nn.Linear(feedforward_dims, in_dims)
        self.drop = nn.Dropout(drop_prob)
        self.act = act_layer()
        if act_layer is not nn.GELU:
            raise NotImplementedError("PreNormFF: GELU only")

    def forward(self, x):
        c = x.shape[-1]
        x2 = x.reshape(-1, c)
        xn, x2 = mf.layer_norm_skip(x2, self.norm.weight, self.norm.bias, self.norm.eps)
        y = mf.mlp(xn, self.lin1.weight, self.lin1.bias, self.lin2.weight, self.lin2.bias, residual=x2,
                   p_mid=self.drop.p, p_out=self.drop.p, training=self.training)
        return y.view(x.shape)


class PreNormDWConvFF(nn.Module):
    """:44-92 x + drop(lin3(GELU(BN(dwconv5x5(GLU(lin1(LN(x)))))))): the depthwise conv pads
    by replication (padding_mode, :65) -- a clamp-gather of the GLU output, the stock
    depthwise kernel on the padded map, and the fold of its gradient on the way back."""

    def __init__(self, in_dims: int, drop_prob: float = 0.0, feedforward_dims: Optional[int] = None,
                 kernel_size: int = 5, act_layer=nn.GELU):
        super().__init__()
        if feedforward_dims is None:
            feedforward_dims = 4 * in_dims
        self.in_dims = in_dims
        self.feedforward_dims = feedforward_dims
        self.norm = nn.LayerNorm(in_dims)
        self.lin1 = nn.Linear(in_dims, feedforward_dims * 2)
        self.act1 = nn.GLU(dim=-1)
        self.kernel_size = kernel_size
        self.conv2 = nn.Conv2d(feedforward_dims, feedforward_dims, kernel_size=(kernel_size, kernel_size), bias=False,
                               stride=(1, 1), padding=(2, 2), padding_mode=_CONV_PADDING_MODE, groups=feedforward_dims)
        self.bn2 = nn.BatchNorm2d(feedforward_dims)
        self.act2 = act_layer()
        self.lin3 = nn.Linear(feedforward_dims, in_dims)
        self.drop = nn.Dropout(drop_prob)
        self.initialize_parameters()
        if act_layer is not nn.GELU:
            raise NotImplementedError("PreNormDWConvFF: GELU only")

    def initialize_parameters(self):
        ks = self.conv2.kernel_size
        nn.init.normal_(self.conv2.weight, mean=0.0, std=math.sqrt(2 / (ks[0] * ks[1])))

    def forward(self, x):
        b, h, w, c = x.shape
        x2 = x.reshape(-1, c)
        xn, x2 = mf.layer_norm_skip(x2, self.norm.weight, self.norm.bias, self.norm.eps)
        g = mf.glu(mf.linear(xn, self.lin1.weight, self.lin1.bias))  # [B*H*W, F]
        g = g.view(b, h, w, self.feedforward_dims)
        p = self.conv2.padding[0]
        g = mf.pad_replicate_nhwc(g, p, p, p, p)
        g = mf.dwconv_nhwc(g, self.conv2.weight, stride=1, same=False, pad=0)
        g = bn_forward(self.bn2, g, L.ACT_GELU)
        if self.drop.p > 0 and self.training:
            y = mf.linear(g.reshape(-1, self.feedforward_dims), self.lin3.weight, self.lin3.bias)
            y = mf.add(mf.dropout(y, self.drop.p, True), x2)
        else:
            y = mf.linear(g.reshape(-1, self.feedforward_dims), self.lin3.weight, self.lin3.bias, residual=x2)
        return y.view(b, h, w, c)
