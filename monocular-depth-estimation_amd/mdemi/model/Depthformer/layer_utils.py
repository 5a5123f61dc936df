"""ConvBN / ResConvBNBlock / UpscaleConcatAct (mirrors model/Depthformer/layer_utils.py) on
libmdemi kernels, NHWC.  ConvBN's conv uses replicate padding (layer_utils.py:18-22): the
implicit-GEMM loader clamps its taps; the backward folds the padded-input gradient back onto
the border pixels (mdemi_pad_fold_replicate)."""
import torch.nn as nn

from ... import _lib as L
from ... import functional as mf
from ..NewCRFs.uper_crf_head import bn_forward


def _act_code(act_layer):
    if act_layer is None:
        return L.ACT_NONE
    if act_layer is nn.SiLU:
        return L.ACT_SILU
    if act_layer is nn.GELU:
        return L.ACT_GELU
    if act_layer is nn.ReLU:
        return L.ACT_RELU
    raise NotImplementedError(f"activation {act_layer}")


class ConvBN(nn.Module):
    """layer_utils.py:6-34: conv (no bias, replicate pad) -> BN -> act (-> + x)."""

    def __init__(self, in_channels, out_channels, kernel_size, act_layer=None, use_residual=True):
        super().__init__()
        if kernel_size % 2 != 1:
            raise ValueError(f"ConvBN kernel size should be odd, got {kernel_size}.")
        self.conv = nn.Conv2d(in_channels, out_channels, bias=False, kernel_size=(kernel_size, kernel_size),
                              stride=(1, 1), padding=(kernel_size // 2, kernel_size // 2), padding_mode="replicate")
        self.bn = nn.BatchNorm2d(out_channels, eps=1e-5)
        self.act = act_layer() if (act_layer is not None) else nn.Identity()
        self._act = _act_code(act_layer)
        self.use_residual = (in_channels == out_channels) and use_residual

    def forward(self, x):
        k = self.conv.kernel_size[0]
        y = mf.conv2d_nhwc(x, self.conv.weight, None, stride=1, pad=k // 2,
                           pad_mode=L.PAD_REPLICATE if k > 1 else L.PAD_ZERO)
        y = bn_forward(self.bn, y, self._act)
        return mf.add(y, x) if self.use_residual else y


class ResConvBNBlock(nn.Module):
    """layer_utils.py:65-99."""

    def __init__(self, in_channels, out_channels, kernel_size, num_layers=2, act_layer=nn.GELU):
        super().__init__()
        self.num_layers = num_layers
        channels = in_channels
        layers = []
        for i in range(num_layers):
            layers.append(ConvBN(channels, out_channels, kernel_size=kernel_size,
                                 act_layer=act_layer if (i != num_layers - 1) else None, use_residual=False))
            channels = out_channels
        self.layers = nn.ModuleList(layers)
        for layer in layers[:-1]:  # each but the last feeds the next layer's conv (bf16 storage)
            layer.bn._mdemi_out_b16 = True
        self.use_residual = (in_channels == out_channels)
        if not self.use_residual:
            self.shortcut = ConvBN(in_channels, out_channels, kernel_size=1, act_layer=None, use_residual=False)
        else:
            self.shortcut = nn.Identity()

    def forward(self, x):
        identity = x
        for layer in self.layers:
            x = layer(x)
        identity = self.shortcut(identity) if not self.use_residual else identity
        return mf.add(x, identity, out_b16=True)  # feeds the 1x1 shoot conv (decoder_v8.py:136)


class UpscaleConcatAct(nn.Module):
    """layer_utils.py:102-122: act(cat([x, up2(y, align_corners=True)]))."""

    def __init__(self, scale_factor, act_layer=nn.GELU):
        super().__init__()
        self.scale_factor = scale_factor
        self.act = act_layer() if (act_layer is not None) else nn.Identity()
        self._act = _act_code(act_layer)

    def forward(self, x_orig_scale, y_to_upscale):
        out = mf.upsample_concat(y_to_upscale, x_orig_scale, scale_factor=self.scale_factor, align_corners=True,
                                 x_first=False)
        return mf.activation(out, self._act)
