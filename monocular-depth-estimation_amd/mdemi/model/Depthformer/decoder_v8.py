"""DepthFormerDecoderV8 (mirrors model/Depthformer/decoder_v8.py:12-171) on libmdemi kernels.

Feature maps are NHWC; aux tokens (B, K, d).  forward() keeps the reference's
contract (bin_width (B, n_bins), bin_cls (B, H/2, W/2, n_bins) softmax
probabilities -- channels-last --, 8 attention maps).  DepthformerV8 calls
parts() instead, which stops at the bin logits and the regressor output so
the bin softmax, the centres and sum_k p_k c_k run as one fused sweep."""
import math
from typing import Optional, Tuple

import torch
import torch.nn as nn

from ... import _lib as L
from ... import functional as mf
from .layer_utils import ConvBN, ResConvBNBlock, UpscaleConcatAct
from .luna_layer import PreNormLunaLayer
from .self_attention import ViTLayer


class DepthFormerDecoderV8(nn.Module):
    def __init__(self, hidden_dim: int, num_heads: int, num_bins: int, num_aux: int, input_channels: Tuple[int, ...],
                 img_size: Tuple[int, int], feedforward_dim: Optional[int] = None, attn_drop_prob: float = 0.1,
                 drop_prob: float = 0.1, act_layer=nn.SiLU):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.num_heads = num_heads
        self.input_channels = input_channels
        self.num_inputs = len(input_channels)
        self.num_bins = num_bins
        self.num_aux = num_aux
        num_layers = self.num_inputs
        self.head_dim = hidden_dim // self.num_heads
        assert self.num_inputs == 5
        self.img_size = img_size
        self.embedding_scale = math.sqrt(1 / hidden_dim)
        self.aux_embedding = nn.Parameter(torch.zeros(1, self.num_aux, hidden_dim))
        nn.init.normal_(self.aux_embedding, mean=0, std=self.embedding_scale)
        self.internal_dims = [hidden_dim // 4, hidden_dim // 4, hidden_dim // 2, hidden_dim // 2, hidden_dim]
        self.internal_heads = [num_heads // 4, num_heads // 4, num_heads // 2, num_heads // 2, num_heads]
        self.luna_layers = nn.ModuleList([
            PreNormLunaLayer(self.internal_dims[i + 1], hidden_dim, self.internal_dims[i + 1],
                             self.internal_heads[i + 1], feedforward_dim=feedforward_dim,
                             attn_drop_prob=attn_drop_prob, drop_prob=drop_prob, act_layer=act_layer)
            for i in range(num_layers - 1)])
        self.aux_layer = ViTLayer(hidden_dim, hidden_dim, num_heads, feedforward_dim=feedforward_dim,
                                  attn_drop_prob=attn_drop_prob, drop_prob=drop_prob, act_layer=act_layer)
        self.post_conv_layers = nn.ModuleList([
            ResConvBNBlock(self.input_channels[i] + self.internal_dims[i + 1], self.internal_dims[i], 3, num_layers=2,
                           act_layer=act_layer)
            for i in range(num_layers - 1)])
        self.post_conv_layers.append(
            ResConvBNBlock(self.input_channels[-1], self.internal_dims[-1], 3, num_layers=2, act_layer=act_layer))
        self.upscale_layers = nn.ModuleList([UpscaleConcatAct(scale_factor=2, act_layer=act_layer)
                                             for _ in range(num_layers - 1)])
        self.shoot_layers = nn.ModuleList([ConvBN(self.internal_dims[i], self.hidden_dim // 8, kernel_size=1,
                                                  act_layer=act_layer) for i in range(num_layers)])
        self.bin_regressor = nn.Sequential(
            nn.Linear(self.hidden_dim, self.hidden_dim), nn.Dropout(drop_prob, inplace=True), act_layer(),
            nn.Linear(self.hidden_dim, self.hidden_dim), nn.Dropout(drop_prob, inplace=True), act_layer(),
            nn.Linear(self.hidden_dim, self.num_bins))
        self.bin_predictor = nn.Sequential(
            ConvBN(self.hidden_dim * 5 // 8, self.hidden_dim, 3, act_layer=act_layer, use_residual=False),
            ConvBN(self.hidden_dim, self.hidden_dim, 3, act_layer=act_layer, use_residual=False),
            nn.Conv2d(self.hidden_dim, self.num_bins, kernel_size=(1, 1)))
        self.bin_predictor[0].bn._mdemi_out_b16 = True  # both feed a conv (bf16 storage)
        self.bin_predictor[1].bn._mdemi_out_b16 = True
        self._act = L.ACT_SILU if act_layer is nn.SiLU else None
        if self._act is None:
            raise NotImplementedError("DepthFormerDecoderV8 runs with its default act_layer=nn.SiLU")

    def parts(self, features):
        """-> (regressor output (B, n_bins), bin logits NHWC (B, H/2, W/2, n_bins), 8 attention maps)."""
        x0, x1, x2, x3, x4 = features
        B, out_h, out_w = x0.shape[0], x0.shape[1], x0.shape[2]
        c4 = self.post_conv_layers[4](x4)
        out4 = self.shoot_layers[4](c4)
        aux = mf.add_rows_broadcast(torch.zeros(B, self.num_aux, self.hidden_dim, device=x0.device),
                                    self.aux_embedding.view(self.num_aux, self.hidden_dim))
        c4, aux, attn4_1, attn4_2 = self.luna_layers[3](c4, aux)
        c3 = self.post_conv_layers[3](self.upscale_layers[3](x3, c4))
        out3 = self.shoot_layers[3](c3)
        c3, aux, attn3_1, attn3_2 = self.luna_layers[2](c3, aux)
        c2 = self.post_conv_layers[2](self.upscale_layers[2](x2, c3))
        out2 = self.shoot_layers[2](c2)
        c2, aux, attn2_1, attn2_2 = self.luna_layers[1](c2, aux)
        c1 = self.post_conv_layers[1](self.upscale_layers[1](x1, c2))
        out1 = self.shoot_layers[1](c1)
        c1, aux, attn1_1, attn1_2 = self.luna_layers[0](c1, aux)
        aux, _ = self.aux_layer(aux)
        c0 = self.post_conv_layers[0](self.upscale_layers[0](x0, c1))
        out0 = self.shoot_layers[0](c0)
        # decoder_v8.py:152-156: x2..x16 bilinear (align_corners=True) resizes written straight into
        # their channel slices of the concatenation
        out = mf.resize_concat([out0, out1, out2, out3, out4], (out_h, out_w), align_corners=True)
        z = self.bin_predictor[1](self.bin_predictor[0](out))
        head = self.bin_predictor[2]
        logits = mf.conv2d_nhwc(z, head.weight, head.bias, stride=1, pad=0)
        a = mf.spatial_mean(aux)                                            # torch.mean(aux, dim=1)
        r = self.bin_regressor
        tr = self.training
        a = mf.activation(mf.dropout(mf.linear(a, r[0].weight, r[0].bias), r[1].p, tr), self._act)
        a = mf.activation(mf.dropout(mf.linear(a, r[3].weight, r[3].bias), r[4].p, tr), self._act)
        raw = mf.linear(a, r[6].weight, r[6].bias)
        attn = (attn1_1, attn1_2, attn2_1, attn2_2, attn3_1, attn3_2, attn4_1, attn4_2)
        return raw, logits, attn

    def forward(self, features):
        raw, logits, attn = self.parts(features)
        bin_width, _, _ = mf.bins_from_raw(raw, L.BINS_ELU, 0.0, 1.0, with_widths=True)
        bin_cls = mf.softmax_lastdim(logits)
        return bin_width, bin_cls, attn
