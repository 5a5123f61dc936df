"""CPU restatement of model/Adabins (everything after the EfficientNet-B5
encoder).  TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.
Pinned by tests/golden/{adabins_head,mvit}.npz.  The encoder itself is a
torch.hub download in the reference (unet_adaptive_bins.py:129): parity unpinned.
"""
import torch
import torch.nn.functional as F

from . import bnmode

# Test hook (kink-aware comparisons): when set to a list of boolean tensors, every
# ReLU / LeakyReLU of the head takes its branch from the next mask in call order
# (mask = "pre-activation > 0" as the GPU forward decided it) instead of from the sign
# of its own input, so the oracle differentiates the same piecewise-linear function as
# the GPU even where an fp32 rounding put a pre-activation on the other side of the kink.
KINK = None


def _kink_act(x, slope):
    """F.relu (slope 0) / F.leaky_relu (slope 0.01), or the KINK-masked branch."""
    global KINK
    if KINK is not None:
        m = KINK.pop(0).to(x.device)
        assert m.shape == x.shape, (m.shape, x.shape)
        return torch.where(m, x, x * slope)
    return F.leaky_relu(x, slope) if slope else F.relu(x)


def bn_train(P, pre, x, eps=1e-5):
    """Batch statistics, or the running ones inside bnmode.eval_bn()."""
    return bnmode.batch_norm(P, pre, x, eps)


def upsample_bn(P, pre, x, concat_with):  # unet_adaptive_bins.py:8-24
    up_x = F.interpolate(x, size=[concat_with.size(2), concat_with.size(3)], mode="bilinear", align_corners=True)
    f = torch.cat([up_x, concat_with], dim=1)
    f = _kink_act(bn_train(P, pre + "_net.1.", F.conv2d(f, P[pre + "_net.0.weight"], P[pre + "_net.0.bias"],
                                                         padding=1)), 0.01)
    return _kink_act(bn_train(P, pre + "_net.4.", F.conv2d(f, P[pre + "_net.3.weight"], P[pre + "_net.3.bias"],
                                                            padding=1)), 0.01)


def decoder_bn(P, pre, features):  # unet_adaptive_bins.py:27-57
    b0, b1, b2, b3, b4 = features[4], features[5], features[6], features[8], features[11]
    x = F.conv2d(b4, P[pre + "conv2.weight"], P[pre + "conv2.bias"], padding=1)
    x = upsample_bn(P, pre + "up1.", x, b3)
    x = upsample_bn(P, pre + "up2.", x, b2)
    x = upsample_bn(P, pre + "up3.", x, b1)
    x = upsample_bn(P, pre + "up4.", x, b0)
    return F.conv2d(x, P[pre + "conv3.weight"], P[pre + "conv3.bias"], padding=1)


def transformer_encoder_layer(P, pre, src, heads):
    """nn.TransformerEncoderLayer(E, heads, 1024) defaults: post-norm, ReLU, (S,N,E) layout."""
    S, N, E = src.shape
    hd = E // heads
    qkv = F.linear(src, P[pre + "self_attn.in_proj_weight"], P[pre + "self_attn.in_proj_bias"])
    q, k, v = qkv.chunk(3, dim=-1)

    def heads_first(t):
        return t.contiguous().view(S, N * heads, hd).transpose(0, 1)

    q, k, v = heads_first(q), heads_first(k), heads_first(v)
    attn = torch.softmax((q @ k.transpose(-2, -1)) / (hd ** 0.5), dim=-1)
    o = (attn @ v).transpose(0, 1).contiguous().view(S, N, E)
    o = F.linear(o, P[pre + "self_attn.out_proj.weight"], P[pre + "self_attn.out_proj.bias"])
    x = F.layer_norm(src + o, (E,), P[pre + "norm1.weight"], P[pre + "norm1.bias"], 1e-5)
    ff = F.linear(_kink_act(F.linear(x, P[pre + "linear1.weight"], P[pre + "linear1.bias"]), 0.0),
                  P[pre + "linear2.weight"], P[pre + "linear2.bias"])
    return F.layer_norm(x + ff, (E,), P[pre + "norm2.weight"], P[pre + "norm2.bias"], 1e-5)


def patch_transformer(P, pre, x, patch_size=16, heads=4, layers=4):  # layers.py:22-31
    emb = F.conv2d(x, P[pre + "embedding_encoder.weight"], P[pre + "embedding_encoder.bias"],
                   stride=patch_size).flatten(2)
    emb = emb + P[pre + "positional_encodings"][:emb.shape[2], :].T.unsqueeze(0)
    t = emb.permute(2, 0, 1)
    for i in range(layers):
        t = transformer_encoder_layer(P, f"{pre}transformer_encoder.layers.{i}.", t, heads)
    return t


def pixel_wise_dot(x, K):  # layers.py:38-43
    n, c, h, w = x.size()
    y = torch.matmul(x.view(n, c, h * w).permute(0, 2, 1), K.permute(0, 2, 1))
    return y.permute(0, 2, 1).view(n, K.shape[1], h, w)


def mvit(P, pre, x, n_query_channels=128, patch_size=16, norm="linear"):  # miniViT.py:25-48
    tgt = patch_transformer(P, pre + "patch_transformer.", x.clone(), patch_size)
    x = F.conv2d(x, P[pre + "embedding_conv.weight"], P[pre + "embedding_conv.bias"], padding=1)
    head, queries = tgt[0, ...], tgt[1:n_query_channels + 1, ...]
    range_maps = pixel_wise_dot(x, queries.permute(1, 0, 2))
    y = _kink_act(F.linear(head, P[pre + "regressor.0.weight"], P[pre + "regressor.0.bias"]), 0.01)
    y = _kink_act(F.linear(y, P[pre + "regressor.2.weight"], P[pre + "regressor.2.bias"]), 0.01)
    y = F.linear(y, P[pre + "regressor.4.weight"], P[pre + "regressor.4.bias"])
    if norm == "linear":
        y = _kink_act(y, 0.0) + 0.1
    elif norm == "softmax":
        return torch.softmax(y, dim=1), range_maps
    else:
        y = torch.sigmoid(y)
    return y / y.sum(dim=1, keepdim=True), range_maps


def bins_to_pred(probs, bin_widths_normed, min_val, max_val):  # unet_adaptive_bins.py:99-107
    bin_widths = (max_val - min_val) * bin_widths_normed
    bin_widths = F.pad(bin_widths, (1, 0), mode="constant", value=min_val)
    bin_edges = torch.cumsum(bin_widths, dim=1)
    centers = 0.5 * (bin_edges[:, :-1] + bin_edges[:, 1:])
    n, dout = centers.size()
    pred = torch.sum(probs * centers.view(n, dout, 1, 1), dim=1, keepdim=True)
    return pred, bin_edges


def adabins_head(P, features, min_val=1e-3, max_val=10.0):  # unet_adaptive_bins.py:93-109 after the encoder
    unet_out = decoder_bn(P, "decoder.", features)
    widths, range_maps = mvit(P, "adaptive_bins_layer.", unet_out)
    probs = torch.softmax(F.conv2d(range_maps, P["conv_out.0.weight"], P["conv_out.0.bias"]), dim=1)
    return bins_to_pred(probs, widths, min_val, max_val)


def unet_adaptive_bins(P, x, min_val=1e-3, max_val=10.0):
    """Whole UnetAdaptiveBins.forward (unet_adaptive_bins.py:93-109) with the restated
    EfficientNet-B5 encoder (oracle/efficientnet.py — parity unpinned)."""
    from . import efficientnet as oeff
    feats = oeff.features(P, "encoder.original_model.", x, last=11)
    return adabins_head(P, feats, min_val, max_val)


def bins_chamfer_loss(bin_edges, target_depth_maps, thresh=1e-3, from_edges=True):
    """AdaBins BinsChamferLoss (upstream AdaBins loss.py; the reference snapshot's loss module is
    absent -- parity unpinned) over pytorch3d.loss.chamfer_distance with its defaults
    (squared L2, point_reduction="mean", batch_reduction="mean"; pytorch3d is not installed, so
    its published definition is restated): per image, x = bin centres (e_i + e_{i+1}) / 2,
    y = target depths >= thresh (the upstream mask `ge(1e-3)`);
    loss = mean_b [ mean_x min_y (x - y)^2 + mean_y min_x (x - y)^2 ].  Differentiable in the
    edges (torch autograd through min / gather), brute force.  from_edges=False takes the
    centres themselves (B, P, ...) (Depthformer v8)."""
    if from_edges:
        centers = 0.5 * (bin_edges[:, 1:] + bin_edges[:, :-1])
    else:
        centers = bin_edges.reshape(bin_edges.shape[0], -1)
    tgt = target_depth_maps.flatten(1)
    total = 0.0
    for c, t in zip(centers, tgt):
        t = t[t >= thresh]
        d = (c[:, None] - t[None, :]) ** 2  # (P, Ny)
        total = total + d.min(dim=1).values.mean() + d.min(dim=0).values.mean()
    return total / centers.shape[0]
