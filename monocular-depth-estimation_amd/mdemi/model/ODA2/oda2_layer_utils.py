"""ConvBN of model/ODA2/oda2_layer_utils.py on libmdemi kernels (NHWC): conv (no bias,
replicate padding -- the implicit-GEMM loader clamps its taps, the backward folds the
padded-input gradient onto the border) -> BatchNorm (or GroupNorm) -> activation fused into
the norm sweep.  Same constructor arguments and attribute names (conv / bn / act)."""
from typing import Optional

import torch.nn as nn

from ... import _lib as L
from ... import functional as mf
from ..Depthformer.layer_utils import _act_code
from ..NewCRFs.uper_crf_head import bn_forward

_CONV_PADDING_MODE = "replicate"


class ConvBN(nn.Module):
    """oda2_layer_utils.py:13-50."""

    def __init__(self, in_ch: int, out_ch: int, kernel_size: int, conv_groups: int = 1, use_gn: bool = False,
                 gn_groups: int = 1, gn_per_group: int = -1, act_layer: Optional = nn.GELU, **act_kwargs):
        super().__init__()
        assert kernel_size % 2 == 1
        if conv_groups != 1:
            raise NotImplementedError("ConvBN: grouped convolution (no ODA2 ordered-swin2 config uses it)")
        if act_kwargs:
            raise NotImplementedError(f"ConvBN: activation arguments {sorted(act_kwargs)}")
        self.in_ch = in_ch
        self.out_ch = out_ch
        self.conv = nn.Conv2d(in_ch, out_ch, kernel_size=(kernel_size, kernel_size), stride=(1, 1),
                              padding=(kernel_size // 2, kernel_size // 2), padding_mode=_CONV_PADDING_MODE,
                              groups=conv_groups, bias=False)
        if (gn_per_group > 0) and use_gn:
            if out_ch % gn_per_group != 0:
                raise ValueError(f"GroupNorm ch {out_ch} not divisible by {gn_per_group}.")
            gn_groups = out_ch // gn_per_group
        self.bn = nn.BatchNorm2d(out_ch) if not use_gn else nn.GroupNorm(gn_groups, out_ch)
        self.act = act_layer() if (act_layer is not None) else nn.Identity()
        self._act = _act_code(act_layer)

    def forward(self, x):
        """x: NHWC."""
        k = self.conv.kernel_size[0]
        y = mf.conv2d_nhwc(x, self.conv.weight, None, stride=1, pad=k // 2,
                           pad_mode=L.PAD_REPLICATE if k > 1 else L.PAD_ZERO)
        if isinstance(self.bn, nn.GroupNorm):
            return mf.group_norm_nhwc(y, self.bn.weight, self.bn.bias, self.bn.num_groups, self.bn.eps, self._act)
        return bn_forward(self.bn, y, self._act)
