"""DepthformerV8 (mirrors model/Depthformer/depthformer_v8.py:27-102) on libmdemi kernels.

forward(x NCHW) -> (depth (B, 1, H/2, W/2), centers (B, n_bins, 1, 1), 8 attention maps) with the
reference's state_dict keys (encoder.backend.*, decoder.*).  The decoder's bin softmax, the
ELU-normalised bin widths -> edges -> centres, and depth = sum_k p_k c_k run as two small
kernels (mdemi_bins_fwd, mdemi_binhead_nhwc_fwd) instead of four ATen passes over the
(B, n_bins, H/2, W/2) probabilities."""
from typing import List

import torch.nn as nn

from ... import _lib as L
from ... import functional as mf
from ..gen_efficientnet import tf_efficientnet_b5_ap, walk_features
from .decoder_v8 import DepthFormerDecoderV8


class Encoder(nn.Module):
    """depthformer_v8.py:10-24 (the walk stops at feature 10, the last one the decoder reads)."""

    def __init__(self, backend: nn.Module):
        super().__init__()
        self.backend = backend

    def forward(self, x, last=10) -> List:
        return walk_features(self.backend, x, last)


class DepthformerV8(nn.Module):
    def __init__(self, backend, opt, min_depth: float, max_depth: float):
        super().__init__()
        self.encoder = Encoder(backend)
        self.decoder = DepthFormerDecoderV8(hidden_dim=opt["hidden_dim"], num_heads=opt["num_heads"],
                                            num_bins=opt["num_bins"], num_aux=opt["num_aux"],
                                            input_channels=(24, 40, 64, 176, 512), img_size=opt["img_size"],
                                            attn_drop_prob=opt.get("attn_drop_prob", 0.1),
                                            drop_prob=opt.get("drop_prob", 0.1))
        self.min_depth = min_depth
        self.max_depth = max_depth

    def forward(self, x):
        f = self.encoder(x)
        raw, logits, attn_weights = self.decoder.parts((f[4], f[5], f[6], f[8], f[10]))
        _, centers = mf.bins_from_raw(raw, L.BINS_ELU, self.min_depth, self.max_depth)
        depth = mf.bin_head_nhwc(logits, centers)
        B, K = centers.shape
        return depth, centers.view(B, K, 1, 1), attn_weights

    def count_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    @classmethod
    def build(cls, opt, min_depth: float, max_depth: float):
        basemodel = tf_efficientnet_b5_ap(pretrained=True)
        del basemodel.conv_head  # depthformer_v8.py:92-96
        del basemodel.bn2
        del basemodel.act2
        del basemodel.global_pool
        del basemodel.classifier
        m = cls(basemodel, opt, min_depth=min_depth, max_depth=max_depth)
        print(f"Model built! #params: {m.count_params()}")
        return m
