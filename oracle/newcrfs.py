"""CPU restatement of model/NewCRFs (Swin backbone, NeW-CRF layers, PSP head,
DispHead).  TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.

Functional form: every function takes P (a name -> tensor dict keyed exactly
like the reference state_dict) and a key prefix.  NCHW / (B, L, C) like the
reference; DropPath is identity (parity runs have stochastic depth off).
Pinned by tests/golden/{swin_*,newcrf_layer,psp_head,disp_head,newcrfs_tiny07}.npz.
"""
import numpy as np
import torch
import torch.nn.functional as F


def window_partition(x, ws):  # swin_transformer.py:32-44
    B, H, W, C = x.shape
    x = x.view(B, H // ws, ws, W // ws, ws, C)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(-1, ws, ws, C)


def window_reverse(windows, ws, H, W):  # swin_transformer.py:47-61
    B = int(windows.shape[0] / (H * W / ws / ws))
    x = windows.view(B, H // ws, W // ws, ws, ws, -1)
    return x.permute(0, 1, 3, 2, 4, 5).contiguous().view(B, H, W, -1)


def relative_position_index(ws):  # swin_transformer.py:91-101
    coords = torch.stack(torch.meshgrid([torch.arange(ws), torch.arange(ws)], indexing="ij"))
    flat = torch.flatten(coords, 1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return rel.sum(-1)


def shift_mask(H, W, ws, shift):  # swin_transformer.py:361-380 / newcrf_layers.py:331-350
    Hp = int(np.ceil(H / ws)) * ws
    Wp = int(np.ceil(W / ws)) * ws
    img_mask = torch.zeros((1, Hp, Wp, 1))
    cnt = 0
    for h in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
        for w in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            img_mask[:, h, w, :] = cnt
            cnt += 1
    mw = window_partition(img_mask, ws).view(-1, ws * ws)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return m.masked_fill(m != 0, float(-100.0)).masked_fill(m == 0, float(0.0))


def _rel_bias(table, ws, heads):
    idx = relative_position_index(ws)
    b = table[idx.view(-1)].view(ws * ws, ws * ws, -1)
    return b.permute(2, 0, 1).contiguous()


def window_attention(P, pre, x, mask, heads, ws):  # swin_transformer.py:112-144
    B_, N, C = x.shape
    qkv = F.linear(x, P[pre + "qkv.weight"], P[pre + "qkv.bias"])
    qkv = qkv.reshape(B_, N, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    q = q * (C // heads) ** -0.5
    attn = q @ k.transpose(-2, -1)
    attn = attn + _rel_bias(P[pre + "relative_position_bias_table"], ws, heads).unsqueeze(0)
    if mask is not None:
        nW = mask.shape[0]
        attn = attn.view(B_ // nW, nW, heads, N, N) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, heads, N, N)
    attn = attn.softmax(-1)
    x = (attn @ v).transpose(1, 2).reshape(B_, N, C)
    return F.linear(x, P[pre + "proj.weight"], P[pre + "proj.bias"])


def mlp(P, pre, x):  # swin_transformer.py:11-29
    x = F.gelu(F.linear(x, P[pre + "fc1.weight"], P[pre + "fc1.bias"]))
    return F.linear(x, P[pre + "fc2.weight"], P[pre + "fc2.bias"])


def ln(P, pre, x, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), P[pre + "weight"], P[pre + "bias"], eps)


def swin_block(P, pre, x, H, W, heads, ws, shift, mask):  # swin_transformer.py:189-246
    B, L, C = x.shape
    shortcut = x
    x = ln(P, pre + "norm1.", x).view(B, H, W, C)
    pad_r = (ws - W % ws) % ws
    pad_b = (ws - H % ws) % ws
    x = F.pad(x, (0, 0, 0, pad_r, 0, pad_b))
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


def patch_merging(P, pre, x, H, W):  # swin_transformer.py:262-289
    B, L, C = x.shape
    x = x.view(B, H, W, C)
    if (H % 2 == 1) or (W % 2 == 1):
        x = F.pad(x, (0, 0, 0, W % 2, 0, H % 2))
    x = torch.cat([x[:, 0::2, 0::2], x[:, 1::2, 0::2], x[:, 0::2, 1::2], x[:, 1::2, 1::2]], -1)
    x = x.view(B, -1, 4 * C)
    x = ln(P, pre + "norm.", x)
    return F.linear(x, P[pre + "reduction.weight"])


def basic_layer(P, pre, x, H, W, depth, heads, ws, downsample):  # swin_transformer.py:353-393
    shift = ws // 2
    mask = shift_mask(H, W, ws, shift)
    for i in range(depth):
        x = swin_block(P, f"{pre}blocks.{i}.", x, H, W, heads, ws, 0 if i % 2 == 0 else shift, mask)
    if downsample:
        return x, H, W, patch_merging(P, pre + "downsample.", x, H, W), (H + 1) // 2, (W + 1) // 2
    return x, H, W, x, H, W


def patch_embed(P, pre, x, patch=4):  # swin_transformer.py:420-436
    _, _, H, W = x.shape
    if W % patch != 0:
        x = F.pad(x, (0, patch - W % patch))
    if H % patch != 0:
        x = F.pad(x, (0, 0, 0, patch - H % patch))
    x = F.conv2d(x, P[pre + "proj.weight"], P[pre + "proj.bias"], stride=patch)
    Wh, Ww = x.size(2), x.size(3)
    x = x.flatten(2).transpose(1, 2)
    x = ln(P, pre + "norm.", x)
    return x.transpose(1, 2).view(-1, x.shape[-1], Wh, Ww)


def swin_transformer(P, pre, x, depths, heads, ws):  # swin_transformer.py:590-615
    x = patch_embed(P, pre + "patch_embed.", x)
    Wh, Ww = x.size(2), x.size(3)
    x = x.flatten(2).transpose(1, 2)
    outs = []
    for i in range(len(depths)):
        x_out, H, W, x, Wh, Ww = basic_layer(P, f"{pre}layers.{i}.", x, Wh, Ww, depths[i], heads[i], ws,
                                             i < len(depths) - 1)
        x_out = ln(P, f"{pre}norm{i}.", x_out)
        outs.append(x_out.view(-1, H, W, x_out.shape[-1]).permute(0, 3, 1, 2).contiguous())
    return tuple(outs)


# ---------------------------------------------------------------------------
# NeW-CRF decoder (newcrf_layers.py)
# ---------------------------------------------------------------------------
def crf_window_attention(P, pre, x, v, mask, heads, ws):  # newcrf_layers.py:110-149
    B_, N, C = x.shape
    qk = F.linear(x, P[pre + "qk.weight"], P[pre + "qk.bias"])
    qk = qk.reshape(B_, N, 2, heads, C // heads).permute(2, 0, 3, 1, 4)
    q, k = qk[0], qk[1]
    q = q * (C // heads) ** -0.5
    attn = q @ k.transpose(-2, -1)
    attn = attn + _rel_bias(P[pre + "relative_position_bias_table"], ws, heads).unsqueeze(0)
    if mask is not None:
        nW = mask.shape[0]
        attn = attn.view(B_ // nW, nW, heads, N, N) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, heads, N, N)
    attn = attn.softmax(-1)
    v = v.view(B_, N, heads, -1).transpose(1, 2)
    x = (attn @ v).transpose(1, 2).reshape(B_, N, C)
    return F.linear(x, P[pre + "proj.weight"], P[pre + "proj.bias"])


def crf_block(P, pre, x, v, H, W, heads, ws, shift, mask):  # newcrf_layers.py:195-257
    B, L, C = x.shape
    shortcut = x
    x = ln(P, pre + "norm1.", x).view(B, H, W, C)
    pad_r = (ws - W % ws) % ws
    pad_b = (ws - H % ws) % ws
    x = F.pad(x, (0, 0, 0, pad_r, 0, pad_b))
    v = F.pad(v, (0, 0, 0, pad_r, 0, pad_b))
    _, Hp, Wp, _ = x.shape
    if shift > 0:
        x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
        v = torch.roll(v, shifts=(-shift, -shift), dims=(1, 2))
    else:
        mask = None
    xw = window_partition(x, ws).view(-1, ws * ws, C)
    vw = window_partition(v, ws)
    vw = vw.view(-1, ws * ws, vw.shape[-1])
    aw = crf_window_attention(P, pre + "attn.", xw, vw, mask, heads, ws).view(-1, ws, ws, C)
    x = window_reverse(aw, ws, Hp, Wp)
    if shift > 0:
        x = torch.roll(x, shifts=(shift, shift), dims=(1, 2))
    if pad_r > 0 or pad_b > 0:
        x = x[:, :H, :W, :].contiguous()
    x = shortcut + x.view(B, H * W, C)
    return x + mlp(P, pre + "mlp.", ln(P, pre + "norm2.", x))


def newcrf(P, pre, x, v, heads, ws=7, depth=2):  # newcrf_layers.py:418-433 (+ BasicCRFLayer :323-363)
    if pre + "proj_x.weight" in P:
        x = F.conv2d(x, P[pre + "proj_x.weight"], P[pre + "proj_x.bias"], padding=1)
    if pre + "proj_v.weight" in P:
        v = F.conv2d(v, P[pre + "proj_v.weight"], P[pre + "proj_v.bias"], padding=1)
    Wh, Ww = x.size(2), x.size(3)
    C = x.size(1)
    x = x.flatten(2).transpose(1, 2)
    v = v.transpose(1, 2).transpose(2, 3)
    shift = ws // 2
    mask = shift_mask(Wh, Ww, ws, shift)
    for i in range(depth):
        x = crf_block(P, f"{pre}crf_layer.blocks.{i}.", x, v, Wh, Ww, heads, ws, 0 if i % 2 == 0 else shift, mask)
    x = ln(P, pre + "norm_crf.", x)
    return x.view(-1, Wh, Ww, C).permute(0, 3, 1, 2).contiguous()


# ---------------------------------------------------------------------------
# PSP head (uper_crf_head.py) with mmcv ConvModule semantics
# ---------------------------------------------------------------------------
def conv_module(P, pre, x, padding=0, bn_eval=False):
    """mmcv ConvModule: conv (bias only without norm) -> BN/GN -> ReLU.  BN uses the batch
    statistics (training) or, with bn_eval, the running statistics (model.eval())."""
    x = F.conv2d(x, P[pre + "conv.weight"], P.get(pre + "conv.bias"), padding=padding)
    if pre + "bn.weight" in P:
        if bn_eval:
            x = F.batch_norm(x, P[pre + "bn.running_mean"], P[pre + "bn.running_var"], P[pre + "bn.weight"],
                             P[pre + "bn.bias"], training=False, eps=1e-5)
        else:
            x = F.batch_norm(x, None, None, P[pre + "bn.weight"], P[pre + "bn.bias"], training=True, eps=1e-5)
    elif pre + "gn.weight" in P:
        x = F.group_norm(x, 256, P[pre + "gn.weight"], P[pre + "gn.bias"], eps=1e-5)
    return F.relu(x)


def psp(P, pre, feats, pool_scales=(1, 2, 3, 6), bn_eval=False):  # uper_crf_head.py:350-364 + PPM :46-58
    x = feats[-1]
    outs = [x]
    for i, s in enumerate(pool_scales):
        y = conv_module(P, f"{pre}psp_modules.{i}.1.", F.adaptive_avg_pool2d(x, s))
        outs.append(F.interpolate(y, size=x.shape[2:], mode="bilinear", align_corners=False))
    return conv_module(P, pre + "bottleneck.", torch.cat(outs, 1), padding=1, bn_eval=bn_eval)


def disp_head(P, pre, x, scale):  # NewCRFDepth.py:151-164,185-188
    x = torch.sigmoid(F.conv2d(x, P[pre + "conv1.weight"], P[pre + "conv1.bias"], padding=1))
    if scale > 1:
        x = F.interpolate(x, scale_factor=scale, mode="bilinear", align_corners=False)
    return x


VERSIONS = {  # NewCRFDepth.py:27-41
    "tiny": dict(embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24]),
    "base": dict(embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32]),
    "large": dict(embed_dim=192, depths=[2, 2, 18, 2], num_heads=[6, 12, 24, 48]),
}


def newcrf_depth(P, imgs, version="large07", max_depth=100.0, bn_eval=False):  # NewCRFDepth.py:123-148
    cfg = VERSIONS[version[:-2]]
    ws = int(version[-2:])
    feats = swin_transformer(P, "backbone.", imgs, cfg["depths"], cfg["num_heads"], ws)
    ppm_out = psp(P, "decoder.", feats, bn_eval=bn_eval)
    e3 = F.pixel_shuffle(newcrf(P, "crf3.", feats[3], ppm_out, 32), 2)
    e2 = F.pixel_shuffle(newcrf(P, "crf2.", feats[2], e3, 16), 2)
    e1 = F.pixel_shuffle(newcrf(P, "crf1.", feats[1], e2, 8), 2)
    e0 = newcrf(P, "crf0.", feats[0], e1, 4)
    return disp_head(P, "disp_head1.", e0, 4) * max_depth
