"""NeW-CRFs depth network on libmdemi kernels (mirrors model/NewCRFs/NewCRFDepth.py).

Public contract kept from the reference: NewCRFDepth(version, inv_depth,
pretrained, frozen_stages, min_depth, max_depth); forward(imgs NCHW) ->
depth (B, 1, H, W); identical state_dict keys.  Inside, every feature map is
NHWC and every op is a gfx950 kernel.
"""
import torch.nn as nn

from ... import functional as mf
from .newcrf_layers import NewCRF
from .swin_transformer import SwinTransformer
from .uper_crf_head import PSP


class NewCRFDepth(nn.Module):
    """NewCRFDepth.py:11-148."""

    def __init__(self, version=None, inv_depth=False, pretrained=None, frozen_stages=-1, min_depth=0.1,
                 max_depth=100.0, **kwargs):
        super().__init__()
        self.inv_depth = inv_depth
        self.with_auxiliary_head = False
        self.with_neck = False
        norm_cfg = dict(type="BN", requires_grad=True)
        window_size = int(version[-2:])
        if version[:-2] == "base":
            embed_dim, depths, num_heads, in_channels = 128, [2, 2, 18, 2], [4, 8, 16, 32], [128, 256, 512, 1024]
        elif version[:-2] == "large":
            embed_dim, depths, num_heads, in_channels = 192, [2, 2, 18, 2], [6, 12, 24, 48], [192, 384, 768, 1536]
        elif version[:-2] == "tiny":
            embed_dim, depths, num_heads, in_channels = 96, [2, 2, 6, 2], [3, 6, 12, 24], [96, 192, 384, 768]
        else:
            raise ValueError(f"unknown NewCRFs version {version}")
        backbone_cfg = dict(embed_dim=embed_dim, depths=depths, num_heads=num_heads, window_size=window_size,
                            ape=False, drop_path_rate=kwargs.get("drop_path_rate", 0.3), patch_norm=True,
                            use_checkpoint=False, frozen_stages=frozen_stages)
        embed_dim = 512
        decoder_cfg = dict(in_channels=in_channels, in_index=[0, 1, 2, 3], pool_scales=(1, 2, 3, 6),
                           channels=embed_dim, dropout_ratio=0.0, num_classes=32, norm_cfg=norm_cfg,
                           align_corners=False)
        self.backbone = SwinTransformer(**backbone_cfg)
        win = 7
        crf_dims = [128, 256, 512, 1024]
        v_dims = [64, 128, 256, embed_dim]
        self.crf3 = NewCRF(input_dim=in_channels[3], embed_dim=crf_dims[3], window_size=win, v_dim=v_dims[3],
                           num_heads=32)
        self.crf2 = NewCRF(input_dim=in_channels[2], embed_dim=crf_dims[2], window_size=win, v_dim=v_dims[2],
                           num_heads=16)
        self.crf1 = NewCRF(input_dim=in_channels[1], embed_dim=crf_dims[1], window_size=win, v_dim=v_dims[1],
                           num_heads=8)
        self.crf0 = NewCRF(input_dim=in_channels[0], embed_dim=crf_dims[0], window_size=win, v_dim=v_dims[0],
                           num_heads=4)
        self.decoder = PSP(**decoder_cfg)
        self.disp_head1 = DispHead(input_dim=crf_dims[0])
        self.up_mode = "bilinear"
        self.min_depth = min_depth
        self.max_depth = max_depth
        self.init_weights(pretrained=pretrained)

    def init_weights(self, pretrained=None):
        print(f"== Load encoder backbone from: {pretrained}")
        self.backbone.init_weights(pretrained=pretrained)
        self.decoder.init_weights()

    def forward(self, imgs):
        feats = self.backbone(imgs)  # NHWC stage maps
        ppm_out = self.decoder(feats)
        e3 = mf.pixel_shuffle_nhwc(self.crf3(feats[3], ppm_out), 2)
        e2 = mf.pixel_shuffle_nhwc(self.crf2(feats[2], e3), 2)
        e1 = mf.pixel_shuffle_nhwc(self.crf1(feats[1], e2), 2)
        e0 = self.crf0(feats[0], e1)
        # disp_head1(e0, 4) * max_depth: the scale is folded into the sigmoid sweep
        # (bilinear resampling is linear, so the order does not change the math)
        depth = self.disp_head1(e0, 4, out_scale=self.max_depth)
        B, H, W, _ = depth.shape
        return depth.view(B, 1, H, W)


class DispHead(nn.Module):
    """NewCRFDepth.py:151-164: conv3x3 -> sigmoid -> x`scale` bilinear (align_corners=False). NHWC."""

    def __init__(self, input_dim=100):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, 1, 3, padding=1)
        self.sigmoid = nn.Sigmoid()

    def forward(self, x, scale, out_scale=1.0):
        y = mf.conv2d_nhwc(x, self.conv1.weight, self.conv1.bias, stride=1, pad=1)
        y = mf.sigmoid_scale(y, out_scale)
        if scale > 1:
            y = mf.interpolate_bilinear(y, scale_factor=scale, align_corners=False)
        return y
