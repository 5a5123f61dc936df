"""Neural window FC-CRF layers on libmdemi kernels (mirrors
model/NewCRFs/newcrf_layers.py; same classes, arguments and state_dict keys).
NHWC in and out; the window partition / roll / pad of x and v are index maps
inside the window-attention kernel; v is zero-padded (newcrf_layers.py:216)."""
import torch.nn as nn

from ... import functional as mf
from .swin_transformer import Mlp, relative_position_index, to_2tuple

import torch


class WindowAttention(nn.Module):
    """newcrf_layers.py:62-149: q,k from the qk Linear of x; v from the coarse prediction."""

    def __init__(self, dim, window_size, num_heads, v_dim, qkv_bias=True, qk_scale=None, attn_drop=0.0,
                 proj_drop=0.0):
        super().__init__()
        self.dim = dim
        self.window_size = to_2tuple(window_size)
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        ws = self.window_size[0]
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) * (2 * ws - 1), num_heads))
        self.register_buffer("relative_position_index", relative_position_index(ws))
        self.qk = nn.Linear(dim, dim * 2, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(v_dim, v_dim)
        self.proj_drop = nn.Dropout(proj_drop)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)

    def attend(self, xn, v2, B, H, W, shift):
        if v2.shape[-1] != self.dim:
            raise ValueError("self.dim != v.shape[-1]")  # newcrf_layers.py:143
        qk = mf.linear(xn, self.qk.weight, self.qk.bias)
        return mf.window_attention(qk, self.qk.bias, v2, None, self.relative_position_bias_table, B, H, W,
                                   self.num_heads, self.window_size[0], shift, self.scale, self.dim, v_off=0)


class CRFBlock(nn.Module):
    """newcrf_layers.py:152-257."""

    def __init__(self, dim, num_heads, v_dim, window_size=7, shift_size=0, mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0, act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.v_dim = v_dim
        self.window_size = window_size
        self.shift_size = shift_size
        self.mlp_ratio = mlp_ratio
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, window_size=to_2tuple(window_size), num_heads=num_heads, v_dim=v_dim,
                                    qkv_bias=qkv_bias, qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path_prob = float(drop_path)
        self.norm2 = norm_layer(v_dim)
        self.mlp = Mlp(in_features=v_dim, hidden_features=int(v_dim * mlp_ratio), act_layer=act_layer, drop=drop)
        self.H = None
        self.W = None

    def forward(self, x, v, mask_matrix=None):
        """x: (B, H*W, C); v: (B, H, W, C) NHWC."""
        B, Lq, C = x.shape
        H, W = self.H, self.W
        assert Lq == H * W, "input feature has wrong size"
        x2 = x.reshape(B * Lq, C)
        v2 = v.reshape(B * Lq, v.shape[-1])
        xn, x2 = mf.layer_norm_skip(x2, self.norm1.weight, self.norm1.bias, self.norm1.eps)
        a = self.attn.attend(xn, v2, B, H, W, self.shift_size)
        x2 = mf.linear(a, self.attn.proj.weight, self.attn.proj.bias, residual=x2)
        xn, x2 = mf.layer_norm_skip(x2, self.norm2.weight, self.norm2.bias, self.norm2.eps)
        x2 = self.mlp(xn, residual=x2)
        return x2.view(B, Lq, self.v_dim)


class BasicCRFLayer(nn.Module):
    """newcrf_layers.py:260-363 (v is shared, unchanged, by both blocks)."""

    def __init__(self, dim, depth, num_heads, v_dim, window_size=7, mlp_ratio=4.0, qkv_bias=True, qk_scale=None,
                 drop=0.0, attn_drop=0.0, drop_path=0.0, norm_layer=nn.LayerNorm, downsample=None,
                 use_checkpoint=False):
        super().__init__()
        self.window_size = window_size
        self.shift_size = window_size // 2
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            CRFBlock(dim=dim, num_heads=num_heads, v_dim=v_dim, window_size=window_size,
                     shift_size=0 if (i % 2 == 0) else window_size // 2, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                     qk_scale=qk_scale, drop=drop, attn_drop=attn_drop,
                     drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path, norm_layer=norm_layer)
            for i in range(depth)])
        if downsample is not None:
            raise NotImplementedError("NewCRF builds BasicCRFLayer without downsampling")
        self.downsample = None

    def forward(self, x, v, H, W):
        for blk in self.blocks:
            blk.H, blk.W = H, W
            x = blk(x, v)
        return x, H, W, x, H, W


class NewCRF(nn.Module):
    """newcrf_layers.py:366-433.  forward(x NHWC, v NHWC) -> NHWC (B, H, W, embed_dim)."""

    def __init__(self, input_dim=96, embed_dim=96, v_dim=64, window_size=7, num_heads=4, depth=2, patch_size=4,
                 in_chans=3, norm_layer=nn.LayerNorm, patch_norm=True):
        super().__init__()
        self.embed_dim = embed_dim
        self.patch_norm = patch_norm
        self.proj_x = nn.Conv2d(input_dim, embed_dim, 3, padding=1) if input_dim != embed_dim else None
        if v_dim != embed_dim:
            self.proj_v = nn.Conv2d(v_dim, embed_dim, 3, padding=1)
        elif embed_dim % v_dim == 0:
            self.proj_v = None
        v_dim = embed_dim
        self.crf_layer = BasicCRFLayer(dim=embed_dim, depth=depth, num_heads=num_heads, v_dim=v_dim,
                                       window_size=window_size, mlp_ratio=4.0, qkv_bias=True, qk_scale=None,
                                       drop=0.0, attn_drop=0.0, drop_path=0.0, norm_layer=norm_layer,
                                       downsample=None, use_checkpoint=False)
        self.add_module("norm_crf", norm_layer(embed_dim))

    def forward(self, x, v):
        if self.proj_x is not None:
            x = mf.conv2d_nhwc(x, self.proj_x.weight, self.proj_x.bias, stride=1, pad=1)
        if self.proj_v is not None:
            v = mf.conv2d_nhwc(v, self.proj_v.weight, self.proj_v.bias, stride=1, pad=1)
        B, H, W, C = x.shape
        x_out, H, W, _, _, _ = self.crf_layer(x.reshape(B, H * W, C), v, H, W)
        out = mf.layer_norm(x_out, self.norm_crf.weight, self.norm_crf.bias, self.norm_crf.eps)
        return out.view(B, H, W, self.embed_dim)
