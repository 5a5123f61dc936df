"""ODA2OrderedSwin2RegModel (model/ODA2/oda2_red_order_swin2.py) on libmdemi kernels.

Constructor arguments, ``build(opt, min_depth, max_depth)`` and the forward contract
``forward(x NCHW) -> (out (B,1,h,w), outs tuple, attn_weights tuple)`` follow the
reference; state_dict keys match (encoder.*, decoder.*).  The input is resized to the
reference's fixed sizes (KITTI 448x896 / 448x1536, NYU 448x672; :65-88) with one bilinear
sweep (align_corners=True), the Swin-L/B encoder runs with replicate padding and (in
training, as configured) activation checkpointing, the decoder predicts num_repeats + 1
sigmoid maps at 1/4 of the resized input, each scaled by max_depth.

Deviation, stated: the reference constructor loads the ImageNet-22k Swin checkpoint from
"checkpoint/swin_{base,large}_patch4_window7_224_22k.pth" (:38-41) and fails without it.
Here ``pretrained`` names that file (default None: random init, as every throughput run in
this build uses); ``use_checkpoint`` and ``path_drop_prob`` default to the reference's
hard-coded True / 0.2 and can be overridden (parity tests switch stochastic depth off)."""
from typing import Optional, Tuple

import torch
import torch.nn as nn

from ... import functional as mf
from .oda2_red_order_swin2_decoder import OrderedSwin2RegDecoder
from .oda2_swin_transformer import SwinTransformer

ENCODERS = {"base": dict(embed_dim=128, num_heads=(4, 8, 16, 32)), "B": dict(embed_dim=128, num_heads=(4, 8, 16, 32)),
            "large": dict(embed_dim=192, num_heads=(6, 12, 24, 48)), "L": dict(embed_dim=192, num_heads=(6, 12, 24, 48))}


class ODA2OrderedSwin2RegModel(nn.Module):

    def __init__(self, dec_dim: int, min_depth: float, max_depth: float, num_heads: int, num_repeats: int,
                 num_emb: int, window_size: int = 8, encoder_type: str = "large", output_scale: int = 4,
                 drop_prob: float = 0.0, attn_drop_prob: float = 0.0, bias_type: str = "depth",
                 bias_init: str = "linear", neck_type: str = "red", *, pretrained: Optional[str] = None,
                 use_checkpoint: bool = True, path_drop_prob: float = 0.2, encoder_kwargs: Optional[dict] = None):
        super().__init__()
        if encoder_type not in ENCODERS:
            raise ValueError(f"Unsupported SwinTransformer type {encoder_type}.")
        swin_kwargs = dict(pretrain_img_size=224, patch_size=4, depths=(2, 2, 18, 2), window_size=7,
                           drop_prob=0.0, attn_drop_prob=0.0, path_drop_prob=path_drop_prob,
                           use_checkpoint=use_checkpoint)
        swin_kwargs.update(ENCODERS[encoder_type])
        if encoder_kwargs:  # test harness: a narrower encoder of the same class
            swin_kwargs.update(encoder_kwargs)
        swin = SwinTransformer(**swin_kwargs)
        swin.init_weights(pretrained=pretrained)
        self.encoder = swin
        self.decoder = OrderedSwin2RegDecoder(
            dec_dim, enc_dims=swin.num_features, num_heads=num_heads, num_repeats=num_repeats, num_emb=num_emb,
            window_size=window_size, attn_drop_prob=attn_drop_prob, drop_prob=drop_prob, output_scale=output_scale,
            bias_type=bias_type, bias_init=bias_init, neck_type=neck_type)
        self.min_depth = min_depth
        self.max_depth = max_depth
        self.num_repeats = num_repeats

    def target_size(self, h: int, w: int) -> Tuple[int, int]:
        """:67-86 (asserts as the reference does)."""
        if self.max_depth > 40:  # kitti
            assert h == 352
            assert (w == 704) or (w == 1216)
            return 448, (896 if (w == 704) else 1536)
        assert h == 480
        assert w == 640
        return 448, 672

    def forward(self, x):
        _, _, h, w = x.shape
        nh, nw = self.target_size(h, w)
        x = mf.resize_nchw_no_grad(x, nh, nw, align_corners=True)
        features = self.encoder(x)
        outs, attn_weights = self.decoder(features, scale=self.max_depth)  # sigmoid x max_depth fused
        return outs[-1], outs, attn_weights

    @classmethod
    def build(cls, opt, min_depth: float, max_depth: float, **kwargs):
        """:98-118 (opt = the config's "model" section)."""
        m = cls(dec_dim=opt["dec_dim"], num_heads=opt["num_heads"], num_repeats=opt["num_repeats"],
                num_emb=opt["num_emb"], window_size=opt.get("window_size", 8), min_depth=min_depth,
                max_depth=max_depth, encoder_type=opt["encoder_type"], output_scale=opt.get("output_scale", 4),
                drop_prob=opt.get("drop_prob", 0.0), attn_drop_prob=opt.get("attn_drop_prob", 0.0),
                bias_type=opt.get("bias_type", "depth"), bias_init=opt.get("bias_init", "linear"),
                neck_type=opt.get("neck_type", "red"), **kwargs)
        return m

    def count_params(self) -> int:
        return sum(p.numel() for p in self.parameters())
