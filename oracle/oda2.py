"""CPU restatement of the ODA2 ordered-swin2 family (model/ODA2/oda2_swin_transformer.py,
oda2_layer_utils.py, oda2_red_order_reg_decoder.py, oda2_red_order_swin2_decoder.py,
oda2_red_order_swin2.py).  TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.

Functional form over P (name -> tensor, keyed like the reference state_dict); NCHW /
(B, L, C) like the reference; DropPath is identity (parity runs have stochastic depth off).
The reference's padding quirks are restated as they run (each is F.pad with a 6-tuple on a
4-D tensor, which pads the last three dims):
  * windows: replicate pad of the normed map on the right/bottom (:254-258);
  * PatchMerging: pad tuple (0,0, 0,H%2, 0,W%2) on (B,H,W,C) -- W grows by H%2 and H by
    W%2 (:325-327), so odd sizes only work when H and W have the same parity;
  * PatchEmbed: (0,0, 0,pad_r, 0,pad_b) on NCHW -- H grows by the W remainder and C by the
    H remainder (:487-491), so only H % 4 == 0 runs (the stride-4 conv then floors W).
The reducer head's depth-ordering indices are a floor of a sigmoid (:247-253): callers may
pass `indices` (one tensor per repeat) to evaluate the rest of the graph at given indices,
e.g. the ones a GPU run produced, when a value sits on a floor boundary.
Pinned by tests/golden/oda2_*.npz (tests/golden/make_golden_oda2.py).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from .newcrfs import _rel_bias, ln, mlp, window_partition, window_reverse


# ---------------------------------------------------------------------------
# Swin encoder with replicate padding (oda2_swin_transformer.py)
# ---------------------------------------------------------------------------
def shift_mask(H, W, ws, shift):  # oda2_swin_transformer.py:409-432
    Hp = int(np.ceil(H / ws)) * ws
    Wp = int(np.ceil(W / ws)) * ws
    img_mask = torch.zeros((1, Hp, Wp, 1))
    cnt = 0
    sl = (slice(0, -ws), slice(-ws, -shift), slice(-shift, None))
    for h in sl:
        for w in sl:
            img_mask[:, h, w, :] = cnt
            cnt += 1
    mw = window_partition(img_mask, ws).reshape(-1, ws * ws)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return m.masked_fill(m != 0, float(-100.0)).masked_fill(m == 0, float(0.0))


def window_attention(P, pre, x, mask, heads, ws):  # oda2_swin_transformer.py:149-183
    B_, N, C = x.shape
    qkv = F.linear(x, P[pre + "qkv.weight"], P[pre + "qkv.bias"])
    qkv = qkv.reshape(B_, N, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    q = q * math.sqrt(1 / (C // heads))
    attn = q @ k.transpose(-2, -1)
    attn = attn + _rel_bias(P[pre + "relative_position_bias_table"], ws, heads).unsqueeze(0)
    if mask is not None:
        nW = mask.shape[0]
        attn = attn.view(B_ // nW, nW, heads, N, N) + mask.to(attn.dtype).unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, heads, N, N)
    attn = attn.softmax(-1)
    x = (attn @ v).transpose(1, 2).reshape(B_, N, C)
    return F.linear(x, P[pre + "proj.weight"], P[pre + "proj.bias"])


def swin_block(P, pre, x, H, W, heads, ws, shift, mask):  # oda2_swin_transformer.py:237-295
    B, L, C = x.shape
    shortcut = x
    x = ln(P, pre + "norm1.", x).view(B, H, W, C)
    pad_r = (ws - W % ws) % ws
    pad_b = (ws - H % ws) % ws
    x = F.pad(x, (0, 0, 0, pad_r, 0, pad_b), mode="replicate")
    _, Hp, Wp, _ = x.shape
    if shift > 0:
        x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
    else:
        mask = None
    xw = window_partition(x, ws).view(-1, ws * ws, C)
    aw = window_attention(P, pre + "attn.", xw, mask, heads, ws).view(-1, ws, ws, C)
    x = window_reverse(aw, ws, Hp, Wp)
    if shift > 0:
        x = torch.roll(x, shifts=(shift, shift), dims=(1, 2))
    if pad_r > 0 or pad_b > 0:
        x = x[:, :H, :W, :].contiguous()
    x = shortcut + x.view(B, H * W, C)
    return x + mlp(P, pre + "mlp.", ln(P, pre + "norm2.", x))


def patch_merging(P, pre, x, H, W):  # oda2_swin_transformer.py:311-339
    B, L, C = x.shape
    x = x.view(B, H, W, C)
    if (H % 2 == 1) or (W % 2 == 1):
        x = F.pad(x, (0, 0, 0, H % 2, 0, W % 2), mode="replicate")
    x = torch.cat([x[:, 0::2, 0::2], x[:, 1::2, 0::2], x[:, 0::2, 1::2], x[:, 1::2, 1::2]], -1)
    x = x.view(B, -1, 4 * C)
    return F.linear(ln(P, pre + "norm.", x), P[pre + "reduction.weight"])


def stage(P, pre, x, H, W, depth, heads, ws, downsample):  # oda2_swin_transformer.py:400-452
    shift = ws // 2
    mask = shift_mask(H, W, ws, shift)
    for i in range(depth):
        x = swin_block(P, f"{pre}blocks.{i}.", x, H, W, heads, ws, 0 if i % 2 == 0 else shift, mask)
    if downsample:
        return x, H, W, patch_merging(P, pre + "downsample.", x, H, W), (H + 1) // 2, (W + 1) // 2
    return x, H, W, x, H, W


def patch_embed(P, pre, x, patch=4):  # oda2_swin_transformer.py:482-500
    _, _, h, w = x.shape
    if h % patch != 0 or w % patch != 0:
        pad_r = (patch - w % patch) % patch
        pad_b = (patch - h % patch) % patch
        x = F.pad(x, (0, 0, 0, pad_r, 0, pad_b), mode="replicate")
    x = F.conv2d(x, P[pre + "proj.weight"], P[pre + "proj.bias"], stride=patch)
    wh, ww = x.size(2), x.size(3)
    x = ln(P, pre + "norm.", x.flatten(2).transpose(1, 2))
    return x.transpose(1, 2).reshape(-1, x.shape[-1], wh, ww)


def swin_transformer(P, pre, x, depths, heads, ws=7):  # oda2_swin_transformer.py:658-685
    x = patch_embed(P, pre + "patch_embed.", x)
    B, _, wh, ww = x.shape
    x = x.flatten(2).transpose(1, 2)
    outs = []
    for i in range(len(depths)):
        x_out, H, W, x, wh, ww = stage(P, f"{pre}layers.{i}.", x, wh, ww, depths[i], heads[i], ws,
                                       i < len(depths) - 1)
        x_out = ln(P, f"{pre}norm{i}.", x_out)
        outs.append(x_out.view(B, H, W, -1).permute(0, 3, 1, 2).contiguous())
    return tuple(outs)


# ---------------------------------------------------------------------------
# decoder pieces
# ---------------------------------------------------------------------------
def conv_bn(P, pre, x, k):  # oda2_layer_utils.py:13-50 (replicate pad, no bias, BN train, GELU)
    p = k // 2
    if p:
        x = F.pad(x, (p, p, p, p), mode="replicate")
    x = F.conv2d(x, P[pre + "conv.weight"])
    x = F.batch_norm(x, None, None, P[pre + "bn.weight"], P[pre + "bn.bias"], training=True, eps=1e-5)
    return F.gelu(x)


def up(x, s):  # nn.UpsamplingBilinear2d(scale_factor=s): align_corners=True
    return F.interpolate(x, scale_factor=s, mode="bilinear", align_corners=True) if s != 1 else x


def dwconv_ff(P, pre, x):  # oda2_red_order_reg_decoder.py:44-92 PreNormDWConvFF
    identity = x
    x = F.linear(ln(P, pre + "norm.", x), P[pre + "lin1.weight"], P[pre + "lin1.bias"])
    x = F.glu(x, dim=-1)
    x = x.permute(0, 3, 1, 2)
    x = F.conv2d(F.pad(x, (2, 2, 2, 2), mode="replicate"), P[pre + "conv2.weight"], groups=x.shape[1])
    x = F.batch_norm(x, None, None, P[pre + "bn2.weight"], P[pre + "bn2.bias"], training=True, eps=1e-5)
    x = F.gelu(x).permute(0, 2, 3, 1)
    x = F.linear(x, P[pre + "lin3.weight"], P[pre + "lin3.bias"])
    return x + identity


def ordered_sa(P, pre, x, indices, heads, ws, shift, num_emb, bias_type="depth"):
    """oda2_red_order_swin2_decoder.py:76-132 PreNormOrderedSwinSA.forward -> (out, attn)."""
    b, h, w, d = x.shape
    r = ws
    identity = x
    if shift > 0:
        x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
        indices = torch.roll(indices, shifts=(-shift, -shift), dims=(1, 2))
    de = 0
    if bias_type == "depth":
        iw = window_partition(indices.unsqueeze(-1), r)
        rel = iw.reshape(-1, r * r, 1) - iw.reshape(-1, 1, r * r) + (num_emb - 1)
        de = F.embedding(rel, P[pre + "depth_embedding"]).permute(0, 3, 1, 2)
    xw = window_partition(x, r)
    xn = ln(P, pre + "norm.", xw)

    def heads4(t):
        return t.reshape(-1, r * r, heads, d // heads).transpose(1, 2)

    q = heads4(F.linear(xn, P[pre + "q_proj.weight"], P[pre + "q_proj.bias"]))
    k = heads4(F.linear(xn, P[pre + "k_proj.weight"], P[pre + "k_proj.bias"]))
    v = heads4(F.linear(xn, P[pre + "v_proj.weight"], P[pre + "v_proj.bias"]))
    attn = (q @ k.transpose(-1, -2)) * math.sqrt(1 / (d // heads))
    attn = torch.softmax(attn + de, dim=-1)
    out = (attn @ v).transpose(1, 2).reshape(-1, r, r, d)
    out = F.linear(out, P[pre + "o_proj.weight"], P[pre + "o_proj.bias"])
    out = window_reverse(out, r, h, w)
    if shift > 0:
        out = torch.roll(out, shifts=(shift, shift), dims=(1, 2))
    return out + identity, attn


def ordered_block(P, pre, x, indices, heads, ws, num_emb, bias_type):  # :167-181 OrderedSwinBlock
    x, a1 = ordered_sa(P, pre + "sa1.", x, indices, heads, ws, 0, num_emb, bias_type)
    x = dwconv_ff(P, pre + "ff1.", x)
    x, a2 = ordered_sa(P, pre + "sa2.", x, indices, heads, ws, ws // 2, num_emb, bias_type)
    x = dwconv_ff(P, pre + "ff2.", x)
    x = F.linear(x, P[pre + "linear.weight"])
    return ln(P, pre + "norm.", x), (a1, a2)


def conv_head(P, pre, x, output_scale=4, last=False):  # :209-234 conv_layers[i]
    o = 1 if (last and output_scale == 2) else 0
    if o:
        x = up(x, 2)
    x = conv_bn(P, f"{pre}{o}.", x, 3)
    x = conv_bn(P, f"{pre}{o + 1}.", x, 3)
    return F.conv2d(x, P[f"{pre}{o + 2}.weight"])


def logit_to_indices(logit, num_emb):  # :247-253
    return torch.floor(torch.sigmoid(logit.detach()) * num_emb - 1e-3).long().squeeze(1)


def reg_head(P, pre, x, heads, num_repeats, num_emb, ws, output_scale=4, bias_type="depth", indices=None):
    """:255-281 OrderedSwinRegHead.forward -> (outs, attn_weights, used_indices)."""
    outs, attn_w, used = [], (), []
    for i in range(num_repeats):
        logit = conv_head(P, f"{pre}conv_layers.{i}.", x.permute(0, 3, 1, 2))
        outs.append(torch.sigmoid(logit))
        idx = logit_to_indices(logit, num_emb) if indices is None else indices[i]
        used.append(idx)
        x, aws = ordered_block(P, f"{pre}attn_layers.{i}.", x, idx, heads, ws, num_emb, bias_type)
        attn_w += aws
    logit = conv_head(P, f"{pre}conv_layers.{num_repeats}.", x.permute(0, 3, 1, 2), output_scale, last=True)
    outs.append(torch.sigmoid(logit))
    return tuple(outs), attn_w, used


def neck(P, pre, feats, neck_type):  # oda2_red_order_swin2_decoder.py:505-576
    e4, e8, e16, e32 = feats

    def seq(name, x, n_conv, k=3, scale=1):
        for j in range(n_conv):
            x = conv_bn(P, f"{pre}{name}.{j}.", x, k)
        return up(x, scale)

    if neck_type == "red":
        dec = torch.cat([seq("enc_conv4", e4, 3), seq("enc_conv8", e8, 3, scale=2),
                         seq("enc_conv16", e16, 3, scale=4), seq("enc_conv32", e32, 3, scale=8)], 1)
    elif neck_type == "fpn":
        e32 = seq("enc_conv32", e32, 2, scale=2)
        e16 = seq("enc_conv16", torch.cat([e16, e32], 1), 2, scale=2)
        e8 = seq("enc_conv8", torch.cat([e8, e16], 1), 2, scale=2)
        dec = seq("enc_conv4", torch.cat([e4, e8], 1), 2)
    elif neck_type == "segformer":
        def lin(name, x, s):
            return up(F.conv2d(x, P[f"{pre}{name}.0.weight"], P[f"{pre}{name}.0.bias"]), s)
        dec = torch.cat([lin("enc_conv4", e4, 1), lin("enc_conv8", e8, 2), lin("enc_conv16", e16, 4),
                         lin("enc_conv32", e32, 8)], 1)
        dec = conv_bn(P, pre + "enc_fuse.", dec, 1)
    elif neck_type in ("red33", "red33r"):
        dec = torch.cat([seq("enc_conv4", e4, 2), seq("enc_conv8", e8, 2, scale=2),
                         seq("enc_conv16", e16, 2, scale=4), seq("enc_conv32", e32, 2, scale=8)], 1)
        dec = conv_bn(P, pre + "enc_fuse.", dec, 1)
    elif neck_type == "red33res":
        parts = []
        for s, sc in ((4, 1), (8, 2), (16, 4), (32, 8)):
            e = {4: e4, 8: e8, 16: e16, 32: e32}[s]
            res = conv_bn(P, f"{pre}enc_res{s}.", e, 1)
            parts.append(up(seq(f"enc_conv{s}", e, 2) + res, sc))
        dec = conv_bn(P, pre + "enc_fuse.", torch.cat(parts, 1), 1)
    else:
        raise ValueError(neck_type)
    return dec.permute(0, 2, 3, 1)


def decoder(P, pre, feats, heads, num_repeats, num_emb, ws, neck_type="red", output_scale=4, bias_type="depth",
            indices=None):  # :505-580
    dec = neck(P, pre, feats, neck_type)
    dec = ln(P, pre + "dec_norm.", F.linear(dec, P[pre + "dec_linear.weight"]))
    return reg_head(P, pre + "reducer.", dec, heads, num_repeats, num_emb, ws, output_scale, bias_type, indices)


def target_size(h, w, max_depth):  # oda2_red_order_swin2.py:65-88
    if max_depth > 40:
        assert h == 352 and w in (704, 1216)
        return 448, (896 if w == 704 else 1536)
    assert h == 480 and w == 640
    return 448, 672


def oda2_model(P, x, enc, dec, max_depth, indices=None):
    """oda2_red_order_swin2.py:64-96 -> (out, outs, attn_weights, used_indices).
    enc: dict(depths, num_heads); dec: dict(num_heads, num_repeats, num_emb, window_size,
    neck_type, output_scale, bias_type)."""
    _, _, h, w = x.shape
    nh, nw = target_size(h, w, max_depth)
    x = F.interpolate(x, size=(nh, nw), mode="bilinear", align_corners=True)
    feats = swin_transformer(P, "encoder.", x, enc["depths"], enc["num_heads"])
    outs, attn, used = decoder(P, "decoder.", feats, dec["num_heads"], dec["num_repeats"], dec["num_emb"],
                               dec.get("window_size", 8), dec.get("neck_type", "red"), dec.get("output_scale", 4),
                               dec.get("bias_type", "depth"), indices)
    outs = tuple(o * max_depth for o in outs)
    return outs[-1], outs, attn, used
