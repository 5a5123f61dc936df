"""CPU restatement of model/Depthformer v8 (decoder + bin head, after the
EfficientNet-B5 encoder).  TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.
Pinned by tests/golden/depthformer_v8.npz.  act_layer is nn.SiLU
(decoder_v8.py:24); dropout is p=0 for parity.
"""
import math

import torch
import torch.nn.functional as F

from . import bf16emu as E
from . import bnmode


def ln(P, pre, x, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), P[pre + "weight"], P[pre + "bias"], eps)


def lin(P, pre, x):
    return E.linear(x, P[pre + "weight"], P[pre + "bias"])


def conv_bn(P, pre, x, act=True, use_residual=True):  # layer_utils.py:6-34
    w = P[pre + "conv.weight"]
    k = w.shape[-1]
    identity = x
    if k > 1:
        x = F.pad(x, (k // 2, k // 2, k // 2, k // 2), mode="replicate")
    x = E.conv2d(x, w)
    x = bnmode.batch_norm(P, pre + "bn.", x, 1e-5)
    if act:
        x = F.silu(x)
    if use_residual and w.shape[0] == w.shape[1]:
        x = x + identity
    return x


def res_conv_bn_block(P, pre, x, num_layers=2):  # layer_utils.py:65-99
    identity = x
    for i in range(num_layers):
        x = conv_bn(P, f"{pre}layers.{i}.", x, act=(i != num_layers - 1), use_residual=False)
    if pre + "shortcut.conv.weight" in P:
        identity = conv_bn(P, pre + "shortcut.", identity, act=False, use_residual=False)
    return x + identity


def upscale_concat_act(x_orig, y):  # layer_utils.py:102-122
    y = F.interpolate(y, scale_factor=2, mode="bilinear", align_corners=True)
    return F.silu(torch.cat([x_orig, y], dim=1))


def _split_heads(x, heads):  # luna_layer.py:162-166
    b, k, d = x.shape
    return x.view(b, k, heads, -1).transpose(1, 2).contiguous()


def prenorm_luna_block(P, pre, hidden, aux, heads):  # luna_layer.py:181-259
    b, _, d = hidden.shape
    scale = math.sqrt(1.0 / (d // heads))
    aux_n = ln(P, pre + "aux_norm.", aux)
    hidden_n = ln(P, pre + "norm.", hidden)
    q1 = _split_heads(lin(P, pre + "q1_proj.", aux_n), heads)
    k1 = _split_heads(lin(P, pre + "k1_proj.", hidden_n), heads)
    v1 = _split_heads(lin(P, pre + "v1_proj.", hidden_n), heads)
    attn1 = E.matmul(q1, k1.transpose(-2, -1))
    attn1 = torch.softmax(attn1 * scale, dim=-1)
    out1 = E.matmul(attn1, v1).transpose(1, 2).reshape(b, -1, d)
    out1 = lin(P, pre + "o1_proj.", out1)
    aux_out = aux + out1
    out_n = ln(P, pre + "inter_norm.", out1)
    q2 = _split_heads(lin(P, pre + "q2_proj.", hidden_n), heads)
    k2 = _split_heads(lin(P, pre + "k2_proj.", out_n), heads)
    v2 = _split_heads(lin(P, pre + "v2_proj.", out_n), heads)
    attn2 = E.matmul(q2, k2.transpose(-2, -1))
    attn2 = torch.softmax(attn2 * scale, dim=-1)
    out2 = E.matmul(attn2, v2).transpose(1, 2).reshape(b, -1, d)
    out2 = lin(P, pre + "o2_proj.", out2)
    return hidden + out2, aux_out, attn1, attn2


def feed_forward(P, pre, hidden):  # feed_forward.py:29-46
    h = ln(P, pre + "norm.", hidden)
    h = lin(P, pre + "fc2.", F.silu(lin(P, pre + "fc1.", h)))
    return hidden + h


def prenorm_luna_layer(P, pre, hidden, aux, heads):  # luna_layer.py:305-345
    b, d, h, w = hidden.shape
    hidden = hidden.view(b, d, h * w).transpose(1, 2).contiguous()
    hidden, aux, a1, a2 = prenorm_luna_block(P, pre + "luna_attn.", hidden, aux, heads)
    hidden = feed_forward(P, pre + "feed_forward.", hidden)
    return hidden.transpose(1, 2).reshape(b, d, h, w), aux, a1, a2


def self_attention_block(P, pre, hidden, heads):  # self_attention.py:44-88
    b, s, d = hidden.shape
    residual = hidden
    h = ln(P, pre + "norm.", hidden)
    q = _split_heads(lin(P, pre + "query_proj.", h), heads)
    k = _split_heads(lin(P, pre + "key_proj.", h), heads)
    v = _split_heads(lin(P, pre + "value_proj.", h), heads)
    scale = math.sqrt(1.0 / q.shape[-1])
    attn = torch.softmax(E.matmul(q, k.transpose(-2, -1)) * scale, dim=-1)
    o = E.matmul(attn, v).transpose(1, 2).reshape(b, s, -1)
    return lin(P, pre + "out_proj.", o) + residual, attn


def decoder_v8(P, pre, feats, hidden_dim, num_heads, num_aux):  # decoder_v8.py:97-171
    x0, x1, x2, x3, x4 = feats
    b, _, oh, ow = x0.shape
    heads = [num_heads // 4, num_heads // 4, num_heads // 2, num_heads // 2, num_heads]
    c4 = res_conv_bn_block(P, pre + "post_conv_layers.4.", x4)
    out4 = conv_bn(P, pre + "shoot_layers.4.", c4)
    aux = P[pre + "aux_embedding"].expand(b, num_aux, hidden_dim)
    c4, aux, a41, a42 = prenorm_luna_layer(P, pre + "luna_layers.3.", c4, aux, heads[4])
    c3 = res_conv_bn_block(P, pre + "post_conv_layers.3.", upscale_concat_act(x3, c4))
    out3 = conv_bn(P, pre + "shoot_layers.3.", c3)
    c3, aux, a31, a32 = prenorm_luna_layer(P, pre + "luna_layers.2.", c3, aux, heads[3])
    c2 = res_conv_bn_block(P, pre + "post_conv_layers.2.", upscale_concat_act(x2, c3))
    out2 = conv_bn(P, pre + "shoot_layers.2.", c2)
    c2, aux, a21, a22 = prenorm_luna_layer(P, pre + "luna_layers.1.", c2, aux, heads[2])
    c1 = res_conv_bn_block(P, pre + "post_conv_layers.1.", upscale_concat_act(x1, c2))
    out1 = conv_bn(P, pre + "shoot_layers.1.", c1)
    c1, aux, a11, a12 = prenorm_luna_layer(P, pre + "luna_layers.0.", c1, aux, heads[1])
    aux, _ = self_attention_block(P, pre + "aux_layer.self_attn.", aux, num_heads)
    aux = feed_forward(P, pre + "aux_layer.feed_forward.", aux)
    c0 = res_conv_bn_block(P, pre + "post_conv_layers.0.", upscale_concat_act(x0, c1))
    out0 = conv_bn(P, pre + "shoot_layers.0.", c0)
    up = [F.interpolate(o, size=(oh, ow), mode="bilinear", align_corners=True) for o in (out1, out2, out3, out4)]
    out = torch.cat([out0] + up, dim=1)
    z = conv_bn(P, pre + "bin_predictor.0.", out, use_residual=False)
    z = conv_bn(P, pre + "bin_predictor.1.", z, use_residual=False)
    bin_cls = torch.softmax(E.conv2d(z, P[pre + "bin_predictor.2.weight"], P[pre + "bin_predictor.2.bias"]), dim=1)
    a = torch.mean(aux, dim=1)
    a = F.silu(lin(P, pre + "bin_regressor.0.", a))
    a = F.silu(lin(P, pre + "bin_regressor.3.", a))
    bw = lin(P, pre + "bin_regressor.6.", a)
    bw = F.elu(bw, alpha=0.1) + 0.1
    bw = bw / torch.sum(bw, dim=1, keepdim=True)
    return bw, bin_cls, (a11, a12, a21, a22, a31, a32, a41, a42)


def depthformer_v8(P, feats, opt, min_depth, max_depth):  # depthformer_v8.py:46-75 after the encoder
    bw, bin_cls, attn = decoder_v8(P, "decoder.", feats, opt["hidden_dim"], opt["num_heads"], opt["num_aux"])
    bw = (max_depth - min_depth) * bw
    bw = F.pad(bw, (1, 0), mode="constant", value=min_depth)
    edges = torch.cumsum(bw, dim=-1)
    centers = (0.5 * (edges[..., :-1] + edges[..., 1:])).unsqueeze(-1).unsqueeze(-1)
    depth = torch.sum(bin_cls * centers, dim=1, keepdim=True)
    return depth, centers, attn


def depthformer_v8_full(P, x, opt, min_depth, max_depth):
    """Whole DepthformerV8.forward (depthformer_v8.py:46-75) with the restated EfficientNet-B5
    encoder (oracle/efficientnet.py — parity unpinned)."""
    from . import efficientnet as oeff
    f = oeff.features(P, "encoder.backend.", x, last=10)
    return depthformer_v8(P, (f[4], f[5], f[6], f[8], f[10]), opt, min_depth, max_depth)
