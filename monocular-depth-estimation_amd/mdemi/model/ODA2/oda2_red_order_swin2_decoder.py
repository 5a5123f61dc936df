"""OrderedSwin2RegDecoder of model/ODA2/oda2_red_order_swin2_decoder.py on libmdemi kernels.

Same classes, constructor arguments, state_dict keys and forward contracts as the
reference; maps are NHWC throughout (the reference permutes to NCHW around its convs).

PreNormOrderedSwinSA (:13-132) is the hot op: per window of ws x ws tokens (64 or 256) and
head, softmax(scale * q k^T + E[idx_i - idx_j + n - 1]) with E the learned depth embedding
and idx the per-pixel depth index from the previous stage's logit.  It runs as
  window_shuffle (roll + partition, one gather) -> LayerNorm -> one q|k|v GEMM (the three
  projections' weights stacked, [3d, d]) -> batched QK^T (MFMA) -> ordered softmax sweep
  (bias gathered from the per-window index map) -> batched PV -> o_proj -> scatter back
  (window_reverse + roll) fused with the residual add.
The attention probabilities are materialised because the reference returns them
(``attn_weights``)."""
import math
from typing import Optional, Tuple

import torch
import torch.nn as nn

from ... import _lib as L
from ... import functional as mf
from .oda2_layer_utils import ConvBN
from .oda2_red_order_reg_decoder import PreNormDWConvFF
from .oda2_swin_transformer import SwinWindowing


class PreNormOrderedSwinSA(nn.Module):
    """:13-132."""

    def __init__(self, in_dims: int, num_heads: int, num_emb: int, window_size: int = 8, shift_size: int = 0,
                 attn_drop_prob: float = 0.0, drop_prob: float = 0.0, bias_type: str = "depth",
                 bias_init: str = "linear"):
        super().__init__()
        self.in_dims = in_dims
        self.num_heads = num_heads
        if in_dims % num_heads != 0:
            raise ValueError(f"Input dim {in_dims} is not divisible by num_heads {num_heads}.")
        self.head_dim = in_dims // num_heads
        self.norm = nn.LayerNorm(in_dims)
        self.q_proj = nn.Linear(in_dims, in_dims)
        self.k_proj = nn.Linear(in_dims, in_dims)
        self.v_proj = nn.Linear(in_dims, in_dims)
        self.o_proj = nn.Linear(in_dims, in_dims)
        self.attn_scale = math.sqrt(1 / self.head_dim)
        self.drop = nn.Dropout(drop_prob)
        self.attn_drop = nn.Dropout(attn_drop_prob)
        self.window_size = window_size
        self.shift_size = shift_size
        self.windowing = SwinWindowing(window_size=window_size)
        assert (self.window_size == 16) or (self.window_size == 8) or (self.window_size == 4)
        self.num_emb = num_emb
        self.bias_type = bias_type
        if bias_type == "depth":
            if bias_init == "linear":  # :50-58
                with torch.no_grad():
                    de = torch.linspace(1, 2 * num_emb - 1, 2 * num_emb - 1)
                    de -= num_emb
                    de = de.unsqueeze(-1).expand(2 * num_emb - 1, num_heads).contiguous()
                    init = torch.ones(num_heads, dtype=torch.float32).uniform_(0.01, 0.04)
                    de[:num_emb] *= init
                    de[-num_emb:] *= (-init)
            elif bias_init == "random":
                de = torch.zeros(2 * num_emb - 1, num_heads).uniform_(-0.05, 0.05)
            else:
                raise ValueError(f"Unsupported bias init {bias_init}.")
            self.depth_embedding = nn.Parameter(de, requires_grad=True)
        elif bias_type == "none":
            pass
        elif bias_type == "pos":
            raise NotImplementedError  # as the reference (:66-67)
        else:
            raise ValueError(f"Unsupported bias type {bias_type}.")
        if window_size == 4:
            raise NotImplementedError("ordered window attention: 8x8 and 16x16 windows (the configured sizes)")

    def _qkv_weight(self):
        w = torch.cat([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight], 0)
        b = torch.cat([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias], 0)
        return w, b

    def forward(self, x, indices) -> Tuple[torch.Tensor, torch.Tensor]:
        """x: (B, H, W, d) NHWC; indices: (B, H, W) integer depth indices (no gradient).
        Returns (out (B, H, W, d), attn (B*nW, heads, ws^2, ws^2))."""
        b, h, w, d = x.shape
        assert d == self.in_dims
        r = self.window_size
        if h % r or w % r:
            raise ValueError(f"PreNormOrderedSwinSA: a {h}x{w} map does not tile into {r}x{r} windows "
                             "(the reference's window_partition view fails the same way)")
        s = self.shift_size
        T = r * r
        nwin = b * (h // r) * (w // r)
        xw = mf.window_shuffle(x, r, s)  # [nwin*T, d] window-major, rolled by -s
        xn = mf.layer_norm(xw, self.norm.weight, self.norm.bias, self.norm.eps)
        wqkv, bqkv = self._qkv_weight()
        qkv = mf.linear(xn, wqkv, bqkv)  # [nwin*T, 3d]
        if self.bias_type == "depth":
            idx_w = mf.window_indices(indices, r, s)
            table = self.depth_embedding
        else:
            idx_w, table = None, None
        o, attn = mf.ordered_window_attention(qkv, idx_w, table, nwin, T, self.num_heads, self.head_dim,
                                              self.num_emb, self.attn_scale, p=self.attn_drop.p,
                                              training=self.training)
        o = mf.linear(o, self.o_proj.weight, self.o_proj.bias)
        if self.drop.p > 0 and self.training:
            o = mf.dropout(o, self.drop.p, True)
        out = mf.window_unshuffle_add(o, x, r, s)
        return out, attn


class OrderedSwinBlock(nn.Module):
    """:135-181 sa1 -> ff1 -> sa2 (shifted) -> ff2 -> linear -> norm."""

    def __init__(self, in_dims: int, num_heads: int, num_emb: int, window_size: int = 8,
                 feedforward_dims: Optional[int] = None, attn_drop_prob: float = 0.0, drop_prob: float = 0.0,
                 act_layer=nn.GELU, bias_type: str = "depth", bias_init: str = "linear"):
        super().__init__()
        sa_kwargs = dict(window_size=window_size, attn_drop_prob=attn_drop_prob, drop_prob=drop_prob,
                         bias_type=bias_type, bias_init=bias_init)
        ff_kwargs = dict(feedforward_dims=feedforward_dims, drop_prob=drop_prob, act_layer=act_layer)
        self.sa1 = PreNormOrderedSwinSA(in_dims, num_heads, num_emb, shift_size=0, **sa_kwargs)
        self.ff1 = PreNormDWConvFF(in_dims, **ff_kwargs)
        self.sa2 = PreNormOrderedSwinSA(in_dims, num_heads, num_emb, shift_size=window_size // 2, **sa_kwargs)
        self.ff2 = PreNormDWConvFF(in_dims, **ff_kwargs)
        self.linear = nn.Linear(in_dims, in_dims, bias=False)
        self.norm = nn.LayerNorm(in_dims, elementwise_affine=True)

    def forward(self, x, indices):
        x, attn1 = self.sa1(x, indices)
        x = self.ff1(x)
        x, attn2 = self.sa2(x, indices)
        x = self.ff2(x)
        shp = x.shape
        y = mf.linear(x.reshape(-1, shp[-1]), self.linear.weight)
        y = mf.layer_norm(y, self.norm.weight, self.norm.bias, self.norm.eps)
        return y.view(shp), (attn1, attn2)


class _Upsample(nn.UpsamplingBilinear2d):
    """nn.UpsamplingBilinear2d (align_corners=True) on an NHWC map."""

    def forward(self, x):
        return mf.interpolate_bilinear(x, scale_factor=self.scale_factor, align_corners=True)


class _Conv1x1Logit(nn.Conv2d):
    """nn.Conv2d(in, 1, 1x1, bias=False) -> one logit per pixel (NHWC in, NHWC out)."""

    def forward(self, x):
        return mf.conv2d_nhwc(x, self.weight, self.bias)


def _nchw1(y):
    b, h, w, _ = y.shape
    return y.view(b, 1, h, w)


def _seq_forward(seq, x):
    for m in seq:
        x = m(x)
    return x


class OrderedSwinRegHead(nn.Module):
    """:184-281."""

    def __init__(self, in_dims: int, num_heads: int, num_repeats: int, num_emb: int = 128, window_size: int = 8,
                 feedforward_dims: Optional[int] = None, attn_drop_prob: float = 0.0, drop_prob: float = 0.0,
                 output_scale: int = 4, act_layer=nn.GELU, bias_type: str = "depth", bias_init: str = "linear"):
        super().__init__()
        self.in_dims = in_dims
        self.num_repeats = num_repeats
        self.num_emb = num_emb
        if (output_scale != 2) and (output_scale != 4):
            raise ValueError(f"Output scale should be either 2 or 4, got {output_scale}.")
        self.output_scale = output_scale
        conv_kwargs = dict(act_layer=act_layer, use_gn=False)

        def head(up=False):
            mods = [_Upsample(scale_factor=2)] if up else []
            mods += [ConvBN(in_dims, in_dims // 4, 3, **conv_kwargs), ConvBN(in_dims // 4, in_dims // 4, 3, **conv_kwargs),
                     _Conv1x1Logit(in_dims // 4, 1, kernel_size=(1, 1), stride=(1, 1), bias=False)]
            return nn.Sequential(*mods)

        self.conv_layers = nn.ModuleList([head() for _ in range(num_repeats)])
        self.conv_layers.append(head(up=(output_scale == 2)))
        self.attn_layers = nn.ModuleList([
            OrderedSwinBlock(in_dims, num_heads, num_emb, window_size, feedforward_dims=feedforward_dims,
                             attn_drop_prob=attn_drop_prob, drop_prob=drop_prob, act_layer=act_layer,
                             bias_type=bias_type, bias_init=bias_init)
            for _ in range(num_repeats)])
        self.sigmoid = nn.Sigmoid()

    # Validation path: the attention kernels clamp a depth index to [0, num_emb-1]
    # (csrc/oda2.hip) where the reference's F.embedding would raise on the -1 a saturated
    # logit (sigmoid == 0) produces.  With validate_indices set, every out-of-range index is
    # counted on the device (clamped_indices, no host sync) so a test or a debugging run sees
    # what the clamp hid; off by default (two extra sweeps of the index map per layer).
    validate_indices = False

    @torch.no_grad()
    def _logit_to_indices(self, out):
        """:246-253 floor(sigmoid(logit) * n - 1e-3) (one elementwise sweep, then the cast)."""
        assert out.shape[-1] == 1
        s = mf.activation(out.detach(), L.ACT_SIGMOID)
        idx = torch.floor(s * self.num_emb - 1e-3).to(torch.int32).squeeze(-1)
        if self.validate_indices:
            bad = ((idx < 0) | (idx >= self.num_emb)).sum()
            self.clamped_indices = bad if getattr(self, "clamped_indices", None) is None else self.clamped_indices + bad
        return idx

    def forward_logits(self, x):
        """x: (B, H, W, C) -> (logits: num_repeats + 1 maps (B, H', W', 1), attn_weights)."""
        logits = []
        attn_weights = ()
        for i in range(self.num_repeats):
            logit = _seq_forward(self.conv_layers[i], x)
            logits.append(logit)
            indices = self._logit_to_indices(logit)
            x, aws = self.attn_layers[i](x, indices)
            attn_weights += aws
        logits.append(_seq_forward(self.conv_layers[-1], x))
        return logits, attn_weights

    def forward(self, x, scale: float = 1.0):
        """x: (B, H, W, C).  Returns (outs: scale * sigmoid maps (B, 1, H', W'), attn_weights);
        a one-channel NHWC map is already NCHW, so only the view changes."""
        logits, attn_weights = self.forward_logits(x)
        outs = tuple(_nchw1(mf.sigmoid_scale(lg, scale)) for lg in logits)
        return outs, attn_weights


class OrderedSwin2RegDecoder(nn.Module):
    """:284-580."""

    def __init__(self, dec_dim: int = 512, enc_dims: Tuple[int, int, int, int] = (192, 384, 768, 1536),
                 num_heads: int = 8, num_repeats: int = 3, num_emb: int = 128, window_size: int = 8,
                 attn_drop_prob: float = 0.0, drop_prob: float = 0.0, output_scale: int = 4, act_layer=nn.GELU,
                 bias_type: str = "depth", bias_init: str = "linear", neck_type: str = "red"):
        super().__init__()
        self.dec_dim = dec_dim
        self.enc_dims = enc_dims
        assert len(enc_dims) == 4
        if dec_dim % 4 != 0:
            raise ValueError(f"Decoder dim {dec_dim} should be a multiple of 4.")
        ck = dict(act_layer=act_layer, use_gn=False)
        self.neck_type = neck_type
        Up = _Upsample
        if neck_type == "red":
            def red(c_in, s):
                tail = Up(scale_factor=s) if s > 1 else nn.Identity()
                return nn.Sequential(ConvBN(c_in, c_in, 3, **ck), ConvBN(c_in, dec_dim // 4, 3, **ck),
                                     ConvBN(dec_dim // 4, dec_dim // 4, 3, **ck), tail)
            self.enc_conv32 = red(enc_dims[3], 8)
            self.enc_conv16 = red(enc_dims[2], 4)
            self.enc_conv8 = red(enc_dims[1], 2)
            self.enc_conv4 = red(enc_dims[0], 1)
            enc_channels = (dec_dim // 4) * 4
        elif neck_type == "fpn":
            def fpn(c_in, up):
                tail = Up(scale_factor=2) if up else nn.Identity()
                return nn.Sequential(ConvBN(c_in, dec_dim, 3, **ck), ConvBN(dec_dim, dec_dim, 3, **ck), tail)
            self.enc_conv32 = fpn(enc_dims[3], True)
            self.enc_conv16 = fpn(enc_dims[2] + dec_dim, True)
            self.enc_conv8 = fpn(enc_dims[1] + dec_dim, True)
            self.enc_conv4 = fpn(enc_dims[0] + dec_dim, False)
            enc_channels = dec_dim
        elif neck_type == "segformer":
            def seg(c_in, s):
                tail = Up(scale_factor=s) if s > 1 else nn.Identity()
                return nn.Sequential(nn.Conv2d(c_in, dec_dim, kernel_size=(1, 1)), tail)
            self.enc_conv32 = seg(enc_dims[3], 8)
            self.enc_conv16 = seg(enc_dims[2], 4)
            self.enc_conv8 = seg(enc_dims[1], 2)
            self.enc_conv4 = seg(enc_dims[0], 1)
            self.enc_fuse = ConvBN(dec_dim * 4, dec_dim, kernel_size=1, act_layer=act_layer)
            enc_channels = dec_dim
        elif neck_type in ("red33", "red33r"):
            chs = [dec_dim] * 4 if neck_type == "red33" else [min(c, dec_dim) for c in enc_dims]

            def r33(c_in, c, s):
                tail = Up(scale_factor=s) if s > 1 else nn.Identity()
                return nn.Sequential(ConvBN(c_in, c, 3, **ck), ConvBN(c, c, 3, **ck), tail)
            self.enc_conv32 = r33(enc_dims[3], chs[3], 8)
            self.enc_conv16 = r33(enc_dims[2], chs[2], 4)
            self.enc_conv8 = r33(enc_dims[1], chs[1], 2)
            self.enc_conv4 = r33(enc_dims[0], chs[0], 1)
            self.enc_fuse = ConvBN(sum(chs), dec_dim, kernel_size=1, act_layer=act_layer)
            enc_channels = dec_dim
        elif neck_type == "red33res":
            for s, c_in, sc in ((32, enc_dims[3], 8), (16, enc_dims[2], 4), (8, enc_dims[1], 2), (4, enc_dims[0], 1)):
                setattr(self, f"enc_conv{s}", nn.Sequential(ConvBN(c_in, dec_dim, 3, **ck),
                                                             ConvBN(dec_dim, dec_dim, 3, **ck)))
                setattr(self, f"enc_res{s}", ConvBN(c_in, dec_dim, 1, **ck))
                setattr(self, f"enc_up{s}", Up(scale_factor=sc) if sc > 1 else nn.Identity())
            self.enc_fuse = ConvBN(dec_dim * 4, dec_dim, kernel_size=1, act_layer=act_layer)
            enc_channels = dec_dim
        else:
            raise ValueError(f"Unsupported neck type {neck_type}.")
        self.dec_linear = nn.Linear(enc_channels, dec_dim, bias=False)
        self.dec_norm = nn.LayerNorm(dec_dim, elementwise_affine=True)
        self.reducer = OrderedSwinRegHead(dec_dim, num_heads, num_repeats, num_emb=num_emb, window_size=window_size,
                                          attn_drop_prob=attn_drop_prob, drop_prob=drop_prob,
                                          output_scale=output_scale, act_layer=act_layer, bias_type=bias_type,
                                          bias_init=bias_init)
        self.initialize_parameters()

    def initialize_parameters(self):  # :495-503
        for module in self.modules():
            if isinstance(module, nn.Linear):
                nn.init.trunc_normal_(module.weight, mean=0.0, std=0.02)
                if module.bias is not None:
                    nn.init.zeros_(module.bias)
            elif isinstance(module, nn.Conv2d) and (module.bias is not None):
                nn.init.zeros_(module.bias)

    @staticmethod
    def _seg_conv(seq, x):  # segformer neck: 1x1 conv with bias, then the upsample
        y = mf.conv2d_nhwc(x, seq[0].weight, seq[0].bias)
        return seq[1](y)

    def forward(self, enc_features, scale: float = 1.0):
        """enc_features: the encoder's four NHWC maps.  Returns (outs, attn_weights), outs
        = scale * the sigmoid maps (the wrapper's x max_depth fused into the sigmoid)."""
        e4, e8, e16, e32 = enc_features
        nt = self.neck_type
        if nt == "red":
            dec = mf.concat_channels([_seq_forward(self.enc_conv4, e4), _seq_forward(self.enc_conv8, e8),
                                      _seq_forward(self.enc_conv16, e16), _seq_forward(self.enc_conv32, e32)])
        elif nt == "fpn":
            e32 = _seq_forward(self.enc_conv32, e32)
            e16 = _seq_forward(self.enc_conv16, mf.concat_channels([e16, e32]))
            e8 = _seq_forward(self.enc_conv8, mf.concat_channels([e8, e16]))
            dec = _seq_forward(self.enc_conv4, mf.concat_channels([e4, e8]))
        elif nt == "segformer":
            dec = mf.concat_channels([self._seg_conv(self.enc_conv4, e4), self._seg_conv(self.enc_conv8, e8),
                                      self._seg_conv(self.enc_conv16, e16), self._seg_conv(self.enc_conv32, e32)])
            dec = self.enc_fuse(dec)
        elif nt in ("red33", "red33r"):
            dec = mf.concat_channels([_seq_forward(self.enc_conv4, e4), _seq_forward(self.enc_conv8, e8),
                                      _seq_forward(self.enc_conv16, e16), _seq_forward(self.enc_conv32, e32)])
            dec = self.enc_fuse(dec)
        else:  # red33res
            parts = []
            for s, e in ((4, e4), (8, e8), (16, e16), (32, e32)):
                res = getattr(self, f"enc_res{s}")(e)
                y = mf.add(_seq_forward(getattr(self, f"enc_conv{s}"), e), res)
                parts.append(getattr(self, f"enc_up{s}")(y))
            dec = self.enc_fuse(mf.concat_channels(parts))
        shp = dec.shape
        y = mf.linear(dec.reshape(-1, shp[-1]), self.dec_linear.weight)
        y = mf.layer_norm(y, self.dec_norm.weight, self.dec_norm.bias, self.dec_norm.eps)
        return self.reducer(y.view(shp[0], shp[1], shp[2], self.dec_dim), scale)
