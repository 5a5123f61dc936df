"""Swin Transformer backbone on libmdemi kernels.

Mirrors model/NewCRFs/swin_transformer.py: same classes, constructor
arguments and state_dict keys (so reference checkpoints and the
checkpoint/*_rename.py outputs load unchanged).  Differences are internal:
tokens stay token-major/NHWC, pad+roll+window_partition+window_reverse+crop
are index maps inside the window-attention kernel, LayerNorm/Linear/GELU/
residual run as fused gfx950 kernels, and stage outputs are returned NHWC
(the reference permutes them to NCHW at swin_transformer.py:612).
"""
import torch
import torch.nn as nn

from ... import functional as mf


def to_2tuple(x):
    return tuple(x) if isinstance(x, (list, tuple)) else (x, x)


def relative_position_index(ws):  # swin_transformer.py:91-101
    coords = torch.stack(torch.meshgrid([torch.arange(ws), torch.arange(ws)], indexing="ij"))
    flat = torch.flatten(coords, 1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return rel.sum(-1)


class Mlp(nn.Module):
    """fc1 -> GELU -> fc2 (swin_transformer.py:11-29), one fused autograd op
    (functional.mlp: fc1's epilogue applies GELU and also keeps h for gelu')."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)
        if not isinstance(self.act, nn.GELU):
            raise ValueError("Mlp: only the reference's nn.GELU activation is built")

    def forward(self, x, residual=None, drop_scale=None):
        return mf.mlp(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, residual=residual,
                      drop_scale=drop_scale)


class WindowAttention(nn.Module):
    """W-MSA / SW-MSA with relative position bias (swin_transformer.py:64-144)."""

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, qk_scale=None, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.dim = dim
        self.window_size = to_2tuple(window_size)
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        ws = self.window_size[0]
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) * (2 * ws - 1), num_heads))
        self.register_buffer("relative_position_index", relative_position_index(ws))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)

    def attend(self, xn, B, H, W, shift):
        """xn: normed tokens [B*H*W, C] in natural order -> attention output (pre-proj) [B*H*W, C]."""
        qkv = mf.linear(xn, self.qkv.weight, self.qkv.bias)
        C = self.dim
        return mf.window_attention(qkv, self.qkv.bias, qkv, self.qkv.bias, self.relative_position_bias_table, B, H,
                                   W, self.num_heads, self.window_size[0], shift, self.scale, C, v_off=2 * C)


class SwinTransformerBlock(nn.Module):
    """swin_transformer.py:147-246."""

    def __init__(self, dim, num_heads, window_size=7, shift_size=0, mlp_ratio=4.0, qkv_bias=True, qk_scale=None,
                 drop=0.0, attn_drop=0.0, drop_path=0.0, act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        self.mlp_ratio = mlp_ratio
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, window_size=to_2tuple(window_size), num_heads=num_heads, qkv_bias=qkv_bias,
                                    qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path_prob = float(drop_path)
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        self.H = None
        self.W = None

    def forward(self, x, mask_matrix=None):
        """x: (B, H*W, C) contiguous.  The shift mask is evaluated inside the kernel."""
        B, Lq, C = x.shape
        H, W = self.H, self.W
        assert Lq == H * W, "input feature has wrong size"
        x2 = x.reshape(B * Lq, C)
        # layer_norm_skip: (LN(x), x) -- the residual's gradient is summed inside the LN backward
        xn, x2 = mf.layer_norm_skip(x2, self.norm1.weight, self.norm1.bias, self.norm1.eps)
        a = self.attn.attend(xn, B, H, W, self.shift_size)
        p = self.drop_path_prob if self.training else 0.0
        if p == 0.0:
            x2 = mf.linear(a, self.attn.proj.weight, self.attn.proj.bias, residual=x2)
            xn, x2 = mf.layer_norm_skip(x2, self.norm2.weight, self.norm2.bias, self.norm2.eps)
            x2 = self.mlp(xn, residual=x2)
        else:  # DropPath (swin_transformer.py:232,239): the per-sample scale rides in the proj / fc2 epilogues
            s1 = mf.drop_path_scale(B, p, x.device)
            x2 = mf.linear(a, self.attn.proj.weight, self.attn.proj.bias, residual=x2, drop_scale=s1)
            xn, x2 = mf.layer_norm_skip(x2, self.norm2.weight, self.norm2.bias, self.norm2.eps)
            s2 = mf.drop_path_scale(B, p, x.device)
            x2 = self.mlp(xn, residual=x2, drop_scale=s2)
        return x2.view(B, Lq, C)


class PatchMerging(nn.Module):
    """swin_transformer.py:249-289: 2x2 gather (+pad for odd sizes) -> LN(4C) -> Linear 4C->2C."""

    def __init__(self, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = norm_layer(4 * dim)

    def forward(self, x, H, W):
        B, Lq, C = x.shape
        assert Lq == H * W, "input feature has wrong size"
        g = mf.space_to_depth2(x.reshape(B, H, W, C))
        Ho, Wo = g.shape[1], g.shape[2]
        g = mf.layer_norm(g.reshape(-1, 4 * C), self.norm.weight, self.norm.bias, self.norm.eps)
        return mf.linear(g, self.reduction.weight).view(B, Ho * Wo, 2 * C)


class BasicLayer(nn.Module):
    """One Swin stage (swin_transformer.py:292-393)."""

    def __init__(self, dim, depth, num_heads, window_size=7, mlp_ratio=4.0, qkv_bias=True, qk_scale=None, drop=0.0,
                 attn_drop=0.0, drop_path=0.0, norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False):
        super().__init__()
        self.window_size = window_size
        self.shift_size = window_size // 2
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim=dim, num_heads=num_heads, window_size=window_size,
                                 shift_size=0 if (i % 2 == 0) else window_size // 2, mlp_ratio=mlp_ratio,
                                 qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop, attn_drop=attn_drop,
                                 drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                 norm_layer=norm_layer)
            for i in range(depth)])
        self.downsample = downsample(dim=dim, norm_layer=norm_layer) if downsample is not None else None

    def forward(self, x, H, W):
        for blk in self.blocks:
            blk.H, blk.W = H, W
            x = blk(x)
        if self.downsample is not None:
            return x, H, W, self.downsample(x, H, W), (H + 1) // 2, (W + 1) // 2
        return x, H, W, x, H, W


class PatchEmbed(nn.Module):
    """Conv 4x4 stride 4 + LayerNorm (swin_transformer.py:396-436); patchify sweep + GEMM."""

    def __init__(self, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        patch_size = to_2tuple(patch_size)
        self.patch_size = patch_size
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        """x: NCHW image -> NHWC tokens (B, Wh, Ww, C)."""
        y = mf.patch_embed(x, self.proj.weight, self.proj.bias)
        if self.norm is not None:
            y = mf.layer_norm(y, self.norm.weight, self.norm.bias, self.norm.eps)
        return y


class SwinTransformer(nn.Module):
    """swin_transformer.py:439-620.  forward(NCHW image) -> tuple of NHWC stage maps."""

    def __init__(self, pretrain_img_size=224, patch_size=4, in_chans=3, embed_dim=96, depths=[2, 2, 6, 2],
                 num_heads=[3, 6, 12, 24], window_size=7, mlp_ratio=4.0, qkv_bias=True, qk_scale=None, drop_rate=0.0,
                 attn_drop_rate=0.0, drop_path_rate=0.2, norm_layer=nn.LayerNorm, ape=False, patch_norm=True,
                 out_indices=(0, 1, 2, 3), frozen_stages=-1, use_checkpoint=False):
        super().__init__()
        if ape:
            raise NotImplementedError("absolute position embedding (ape=True) is not used by NewCRFDepth")
        self.pretrain_img_size = pretrain_img_size
        self.num_layers = len(depths)
        self.embed_dim = embed_dim
        self.ape = ape
        self.patch_norm = patch_norm
        self.out_indices = out_indices
        self.frozen_stages = frozen_stages
        self.patch_embed = PatchEmbed(patch_size=patch_size, in_chans=in_chans, embed_dim=embed_dim,
                                      norm_layer=norm_layer if patch_norm else None)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths), device="cpu")]
        self.layers = nn.ModuleList()
        for i in range(self.num_layers):
            self.layers.append(BasicLayer(
                dim=int(embed_dim * 2 ** i), depth=depths[i], num_heads=num_heads[i], window_size=window_size,
                mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop_rate, attn_drop=attn_drop_rate,
                drop_path=dpr[sum(depths[:i]):sum(depths[:i + 1])], norm_layer=norm_layer,
                downsample=PatchMerging if (i < self.num_layers - 1) else None, use_checkpoint=use_checkpoint))
        self.num_features = [int(embed_dim * 2 ** i) for i in range(self.num_layers)]
        for i in out_indices:
            self.add_module(f"norm{i}", norm_layer(self.num_features[i]))
        self._freeze_stages()

    def _freeze_stages(self):  # swin_transformer.py:547-562
        if self.frozen_stages >= 0:
            self.patch_embed.eval()
            for p in self.patch_embed.parameters():
                p.requires_grad = False
        if self.frozen_stages >= 2:
            self.pos_drop.eval()
            for i in range(0, self.frozen_stages - 1):
                m = self.layers[i]
                m.eval()
                for p in m.parameters():
                    p.requires_grad = False

    def init_weights(self, pretrained=None):  # swin_transformer.py:564-588
        def _init(m):
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.LayerNorm):
                nn.init.constant_(m.bias, 0)
                nn.init.constant_(m.weight, 1.0)

        self.apply(_init)
        if isinstance(pretrained, str):
            from ...utils.checkpoint import load_backbone_checkpoint
            load_backbone_checkpoint(self, pretrained)
        elif pretrained is not None:
            raise TypeError("pretrained must be a str or None")

    def forward(self, x):
        t = self.patch_embed(x)
        B, Wh, Ww, C = t.shape
        t = t.reshape(B, Wh * Ww, C)
        outs = []
        for i in range(self.num_layers):
            x_out, H, W, t, Wh, Ww = self.layers[i](t, Wh, Ww)
            if i in self.out_indices:
                nl = getattr(self, f"norm{i}")
                o = mf.layer_norm(x_out, nl.weight, nl.bias, nl.eps)
                outs.append(o.view(B, H, W, self.num_features[i]))
        return tuple(outs)

    def train(self, mode=True):
        super().train(mode)
        self._freeze_stages()
        return self
