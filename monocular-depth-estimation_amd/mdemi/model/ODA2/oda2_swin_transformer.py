"""ODA2's Swin Transformer (model/ODA2/oda2_swin_transformer.py) on libmdemi kernels.

Same classes, constructor arguments and state_dict keys as the reference, so its
checkpoints load unchanged.  Differences from the NeW-CRFs Swin (model/NewCRFs) that this
module restates:

  * replicate padding (``_SWIN_PADDING_MODE``, :12) wherever the map is padded:
      - the windows (:254-258): a map whose size is not a multiple of the window is
        padded by a clamp-gather of the normed tokens (mdemi_pad_replicate) and the
        attention runs on the padded map; the output is cropped by the same gather and the
        backward folds the padded gradient onto the edge tokens.  The common shapes (the
        wrapper resizes to 448 x {672, 896}: 112 x 168 / 224 tokens) need no padding and
        take the fused pad-free window-attention path unchanged;
      - PatchMerging (:325-327) and PatchEmbed (:487-491) restate the reference's F.pad
        calls exactly as they execute, 6-tuple quirks included (see each class);
  * ``use_checkpoint`` (:375,442-443): activation checkpointing of each block in training
    (torch.utils.checkpoint, non-reentrant; RNG state is replayed so stochastic depth
    draws the same masks in the recomputation).  It trades recompute FLOPs for memory:
    the reference sets it for 12 GB GPUs (oda2_red_order_swin2.py:35); on a 288 GB
    MI355X the builder can turn it off (model.use_checkpoint in the config);
  * the shift mask is never materialised (the kernel derives the -100 regions from the
    padded size, :409-432).

Stage outputs are returned NHWC (the reference permutes them to NCHW at :681)."""
from typing import Optional, Tuple, Union

import torch
import torch.nn as nn
import torch.utils.checkpoint as checkpoint

from ... import functional as mf
from ..NewCRFs.swin_transformer import relative_position_index

_SWIN_PADDING_MODE = "replicate"


class SwinMLP(nn.Module):
    """:18-38 fc1 -> GELU -> dropout -> fc2 -> dropout (one fused op; dropout in the
    reference's positions)."""

    def __init__(self, in_features: int, hidden_features: int, drop_prob: float = 0.0, act_layer=nn.GELU) -> None:
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, in_features)
        self.drop = nn.Dropout(drop_prob)
        if not isinstance(self.act, nn.GELU):
            raise ValueError("SwinMLP: only the reference's nn.GELU is built")

    def forward(self, x, residual=None, drop_scale=None):
        p = self.drop.p
        return mf.mlp(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, residual=residual,
                      p_mid=p, p_out=p, training=self.training, drop_scale=drop_scale)


class SwinWindowing(nn.Module):
    """:41-92: window_partition / window_reverse live inside the kernels' index maps; the
    module is kept for the module tree (it has no state)."""

    def __init__(self, window_size: int):
        super().__init__()
        self.window_size = window_size
        self.H: Optional[int] = None
        self.W: Optional[int] = None

    def forward(self):
        raise NotImplementedError

    def extra_repr(self):
        return f"window_size={self.window_size}"


class WindowAttention(nn.Module):
    """:95-183 W-MSA / SW-MSA with relative position bias."""

    def __init__(self, dim: int, window_size: Union[int, Tuple[int, int]], num_heads: int, qkv_bias: bool = True,
                 attn_drop_prob: float = 0.0, drop_prob: float = 0.0) -> None:
        super().__init__()
        self.dim = dim
        self.window_size = (window_size, window_size) if isinstance(window_size, int) else window_size
        self.num_heads = num_heads
        if dim % num_heads != 0:
            raise ValueError(f"Dim {dim} is not divisible by num_heads {num_heads}.")
        head_dim = dim // num_heads
        self.attn_scale = (1 / head_dim) ** 0.5
        ws = self.window_size[0]
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) * (2 * self.window_size[1] - 1),
                                                                     num_heads))
        self.register_buffer("relative_position_index", relative_position_index(ws))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim, bias=True)
        self.attn_drop = nn.Dropout(attn_drop_prob)
        self.proj_drop = nn.Dropout(drop_prob)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)
        if attn_drop_prob > 0 or drop_prob > 0:
            raise NotImplementedError("ODA2 Swin: attention / projection dropout (the ODA2 wrapper builds 0.0, "
                                      "oda2_red_order_swin2.py:33)")

    def attend(self, xn, B, H, W, shift):
        """xn: normed tokens [B*H*W, C] of a map whose sides are multiples of the window
        (padding is done by the block) -> attention output before proj."""
        qkv = mf.linear(xn, self.qkv.weight, self.qkv.bias)
        C = self.dim
        return mf.window_attention(qkv, self.qkv.bias, qkv, self.qkv.bias, self.relative_position_bias_table, B, H,
                                   W, self.num_heads, self.window_size[0], shift, self.attn_scale, C, v_off=2 * C)


class SwinTransformerBlock(nn.Module):
    """:186-295."""

    def __init__(self, dim: int, num_heads: int, window_size: int = 7, shift_size: int = 0, mlp_ratio: float = 4.,
                 qkv_bias: bool = True, attn_drop_prob: float = 0.0, drop_prob: float = 0.0,
                 path_drop_prob: float = 0.0, act_layer=nn.GELU) -> None:
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        self.mlp_ratio = mlp_ratio
        if not (0 <= self.shift_size < self.window_size):
            raise ValueError(f"shift_size {shift_size} must in [0, window_size {window_size})")
        self.norm1 = nn.LayerNorm(dim)
        self.attn = WindowAttention(dim, window_size=self.window_size, num_heads=num_heads, qkv_bias=qkv_bias,
                                    attn_drop_prob=attn_drop_prob, drop_prob=drop_prob)
        self.drop_path = nn.Identity()  # stochastic depth is a fused op (path_drop_prob)
        self.path_drop_prob = float(path_drop_prob)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = SwinMLP(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer,
                           drop_prob=drop_prob)
        self.windowing = SwinWindowing(window_size=window_size)
        self.H: Optional[int] = None
        self.W: Optional[int] = None

    def forward(self, x, mask_matrix=None):
        """x: (B, H*W, C).  mask_matrix is accepted for the reference's signature; the shift
        mask is evaluated inside the kernel."""
        b, n, c = x.shape
        h, w = self.H, self.W
        if n != h * w:
            raise ValueError(f"Input shape {tuple(x.shape)} does not match with size ({h}, {w}).")
        ws = self.window_size
        x2 = x.reshape(b * n, c)
        xn, x2 = mf.layer_norm_skip(x2, self.norm1.weight, self.norm1.bias, self.norm1.eps)
        pad_r = (ws - w % ws) % ws
        pad_b = (ws - h % ws) % ws
        if pad_r or pad_b:  # replicate padding of the normed map (:254-258), crop after (:286-287)
            xp = mf.pad_replicate_nhwc(xn.view(b, h, w, c), bottom=pad_b, right=pad_r)
            a = self.attn.attend(xp.view(-1, c), b, h + pad_b, w + pad_r, self.shift_size)
            a = mf.pad_replicate_nhwc(a.view(b, h + pad_b, w + pad_r, c), bottom=-pad_b, right=-pad_r)
            a = a.view(b * n, c)
        else:
            a = self.attn.attend(xn, b, h, w, self.shift_size)
        p = self.path_drop_prob if self.training else 0.0
        if p == 0.0:
            x2 = mf.linear(a, self.attn.proj.weight, self.attn.proj.bias, residual=x2)
            xn, x2 = mf.layer_norm_skip(x2, self.norm2.weight, self.norm2.bias, self.norm2.eps)
            x2 = self.mlp(xn, residual=x2)
        else:  # DropPath: the per-sample scale rides in the proj / fc2 epilogues
            s1 = mf.drop_path_scale(b, p, x.device)
            x2 = mf.linear(a, self.attn.proj.weight, self.attn.proj.bias, residual=x2, drop_scale=s1)
            xn, x2 = mf.layer_norm_skip(x2, self.norm2.weight, self.norm2.bias, self.norm2.eps)
            if self.mlp.drop.p > 0.0:  # output dropout sits between fc2 and the scale: unfused
                br = self.mlp(xn)
                x2 = mf.drop_path_add(x2.view(b, -1), br.view(b, -1), p, True).view(b * n, c)
            else:
                x2 = self.mlp(xn, residual=x2, drop_scale=mf.drop_path_scale(b, p, x.device))
        return x2.view(b, n, c)


class PatchMerging(nn.Module):
    """:298-339.  The odd-size pad is F.pad(x, (0, 0, 0, h % 2, 0, w % 2), mode="replicate")
    on (B, H, W, C): the last three dims are C, W, H, so W grows by h % 2 and H by w % 2 --
    the 2x2 gather only lines up when h and w have the same parity (otherwise the
    reference's torch.cat fails, and so does this)."""

    def __init__(self, dim: int):
        super().__init__()
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = nn.LayerNorm(4 * dim)

    def forward(self, x, h: int, w: int):
        b, n, c = x.shape
        if n != h * w:
            raise ValueError(f"Input {tuple(x.shape)} does not match with size ({h}, {w})")
        x4 = x.reshape(b, h, w, c)
        if (h % 2 == 1) or (w % 2 == 1):
            if h % 2 != w % 2:
                raise RuntimeError(f"PatchMerging: the reference's replicate pad turns {h}x{w} into "
                                   f"{h + w % 2}x{w + h % 2}, whose 2x2 quadrants do not line up "
                                   "(oda2_swin_transformer.py:326-333)")
            x4 = mf.pad_replicate_nhwc(x4, bottom=w % 2, right=h % 2)
        g = mf.space_to_depth2(x4)
        ho, wo = g.shape[1], g.shape[2]
        g = mf.layer_norm(g.reshape(-1, 4 * c), self.norm.weight, self.norm.bias, self.norm.eps)
        return mf.linear(g, self.reduction.weight).view(b, ho * wo, 2 * c)


class SwinTransformerStage(nn.Module):
    """:342-452 one stage (blocks + optional PatchMerging)."""

    def __init__(self, dim: int, depth: int, num_heads: int, window_size: int = 7, mlp_ratio: float = 4.,
                 qkv_bias: bool = True, drop_prob: float = 0.0, attn_drop_prob: float = 0.0,
                 path_drop_prob: Union[float, Tuple[float, ...]] = 0.0, downsample=None, use_checkpoint=False):
        super().__init__()
        self.window_size = window_size
        self.shift_size = window_size // 2
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(
                dim=dim, num_heads=num_heads, window_size=window_size,
                shift_size=0 if (i % 2 == 0) else window_size // 2, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                drop_prob=drop_prob, attn_drop_prob=attn_drop_prob,
                path_drop_prob=path_drop_prob[i] if isinstance(path_drop_prob, (tuple, list)) else path_drop_prob)
            for i in range(depth)])
        self.windowing = SwinWindowing(window_size=window_size)
        self.downsample = downsample(dim=dim) if downsample is not None else None

    def forward(self, x, h: int, w: int):
        for blk in self.blocks:
            blk.H, blk.W = h, w
            if self.use_checkpoint and self.training and torch.is_grad_enabled():
                x = checkpoint.checkpoint(blk, x, use_reentrant=False)
            else:
                x = blk(x)
        if self.downsample is not None:
            return x, h, w, self.downsample(x, h, w), (h + 1) // 2, (w + 1) // 2
        return x, h, w, x, h, w


class PatchEmbed(nn.Module):
    """:455-500.  The reference pads with F.pad(x, (0, 0, 0, pad_r, 0, pad_b)) on an NCHW
    image, i.e. W by 0, H by pad_r (the W remainder) and C by pad_b (the H remainder): an
    image whose height is not a multiple of the patch breaks the conv's channel count, and
    one whose width is not gets pad_r replicated rows at the bottom while the stride-p conv
    floors the width.  Restated as it runs (the ODA2 wrapper always feeds 448 x {672, 896,
    1536}, so neither case occurs in training)."""

    def __init__(self, patch_size: Union[int, Tuple[int, int]] = 4, in_channels: int = 3, embed_dim: int = 96,
                 out_norm: bool = True):
        super().__init__()
        self.patch_size = (patch_size, patch_size) if isinstance(patch_size, int) else tuple(patch_size)
        self.in_channels = in_channels
        self.embed_dim = embed_dim
        self.proj = nn.Conv2d(in_channels, embed_dim, kernel_size=self.patch_size, stride=self.patch_size)
        self.norm = nn.LayerNorm(embed_dim) if out_norm else None

    def forward(self, x):
        """x: NCHW image -> NHWC tokens (B, Wh, Ww, C)."""
        _, _, h, w = x.shape
        ph, pw = self.patch_size
        if (h % ph != 0) or (w % pw != 0):
            pad_r = (pw - w % pw) % pw
            pad_b = (ph - h % ph) % ph
            if pad_b:
                raise RuntimeError(f"PatchEmbed: the reference's pad adds {pad_b} channels to a {h}x{w} image "
                                   "(F.pad 6-tuple on NCHW, oda2_swin_transformer.py:491) and its conv rejects it")
            # rows replicated; the stride-p conv floors both sides
            x = mf.replicate_rows_nchw_no_grad(x, (h + pad_r) - (h + pad_r) % ph, w - w % pw)
        y = mf.patch_embed(x, self.proj.weight, self.proj.bias)
        if self.norm is not None:
            y = mf.layer_norm(y, self.norm.weight, self.norm.bias, self.norm.eps)
        return y


class SwinTransformer(nn.Module):
    """:503-690.  forward(NCHW image) -> tuple of NHWC stage maps."""

    def __init__(self, pretrain_img_size: int = 224, patch_size: int = 4, in_channels: int = 3, embed_dim: int = 96,
                 depths: Tuple[int, ...] = (2, 2, 6, 2), num_heads: Tuple[int, ...] = (3, 6, 12, 24),
                 window_size: int = 7, mlp_ratio: float = 4.0, qkv_bias: bool = True, drop_prob: float = 0.0,
                 attn_drop_prob: float = 0.0, path_drop_prob: float = 0.2, ape: bool = False,
                 patch_norm: bool = True, out_indices: Tuple[int, ...] = (0, 1, 2, 3), frozen_stages: int = -1,
                 use_checkpoint: bool = False):
        super().__init__()
        if ape:
            raise NotImplementedError("absolute position embedding (ape=True) is not used by the ODA2 wrapper")
        self.pretrain_img_size = pretrain_img_size
        self.num_layers = len(depths)
        self.embed_dim = embed_dim
        self.ape = ape
        self.patch_norm = patch_norm
        self.out_indices = out_indices
        self.frozen_stages = frozen_stages
        self.patch_embed = PatchEmbed(patch_size, in_channels, embed_dim=embed_dim, out_norm=patch_norm)
        self.pos_drop = nn.Dropout(p=drop_prob)
        pdp = [x.item() for x in torch.linspace(0, path_drop_prob, sum(depths), device="cpu")]
        self.layers = nn.ModuleList()
        for i in range(self.num_layers):
            self.layers.append(SwinTransformerStage(
                dim=int(embed_dim * 2 ** i), depth=depths[i], num_heads=num_heads[i], window_size=window_size,
                mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, drop_prob=drop_prob, attn_drop_prob=attn_drop_prob,
                path_drop_prob=tuple(pdp[sum(depths[:i]):sum(depths[:i + 1])]),
                downsample=PatchMerging if (i < self.num_layers - 1) else None, use_checkpoint=use_checkpoint))
        self.num_features = tuple(int(embed_dim * 2 ** i) for i in range(self.num_layers))
        for i in out_indices:
            self.add_module(f"norm{i}", nn.LayerNorm(self.num_features[i]))
        self._freeze_stages()

    def _freeze_stages(self):  # :608-623
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

    @torch.no_grad()
    def init_weights(self, pretrained: Optional[str] = None) -> None:
        """:625-656: trunc_normal(0.02) Linear weights, zero biases; then the Swin
        checkpoint (``model`` key; norm/head/attn_mask entries dropped, the out-norms
        reset to identity), loaded strictly.  pretrained=None keeps the random init (the
        reference requires a path; its files are not in this build)."""
        def _init(m):
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

        self.apply(_init)
        if pretrained is None:
            return
        if not isinstance(pretrained, str):
            raise TypeError(f"Pretrained path should be string, got {pretrained}.")
        sd = torch.load(pretrained, map_location="cpu", weights_only=True)["model"]
        new = {k: v for k, v in sd.items()
               if k not in ("norm.weight", "norm.bias", "head.weight", "head.bias") and "attn_mask" not in k}
        for i in self.out_indices:
            new[f"norm{i}.weight"] = getattr(self, f"norm{i}").weight.data.fill_(1.0)
            new[f"norm{i}.bias"] = getattr(self, f"norm{i}").bias.data.fill_(0.0)
        self.load_state_dict(new, strict=True)

    def forward(self, x):
        t = self.patch_embed(x)
        b, wh, ww, c = t.shape
        t = t.reshape(b, wh * ww, c)
        if self.pos_drop.p > 0 and self.training:
            t = mf.dropout(t, self.pos_drop.p, True)
        outs = []
        for i in range(self.num_layers):
            x_out, h, w, t, wh, ww = self.layers[i](t, wh, ww)
            if i in self.out_indices:
                nl = getattr(self, f"norm{i}")
                o = mf.layer_norm(x_out, nl.weight, nl.bias, nl.eps)
                outs.append(o.view(b, h, w, self.num_features[i]))
        return tuple(outs)

    def train(self, mode=True):
        super().train(mode)
        self._freeze_stages()
        return self
