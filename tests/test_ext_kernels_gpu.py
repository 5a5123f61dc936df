"""Kernel-level numerics of the AdaBins / Depthformer-v8 / EfficientNet-B5 /
evaluation ops (include/mdemi_ext.h) against plain PyTorch fp64 CPU references
of the same op, forward and backward.  fp32 kernels on O(1) data: ~1e-5
relative unless a test states otherwise."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(*shape, generator=g, dtype=torch.float64) * 2 - 1) * scale


def close(a, b, rtol=2e-5, atol=2e-5):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    assert a.shape == b.shape, f"shape {tuple(a.shape)} vs {tuple(b.shape)}"
    err = (a - b).abs().max().item() if a.numel() else 0.0
    ref = b.abs().max().item() if b.numel() else 0.0
    assert err <= atol + rtol * ref, f"max|diff|={err:.3e} max|ref|={ref:.3e}"


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


@pytest.fixture(scope="module")
def mf():
    from mdemi import _lib
    from mdemi import functional as mf
    _lib.load()
    return mf


def tf_same_ref(x, w, stride, groups):
    """gen-efficientnet Conv2dSame: pad (total//2, total - total//2) per axis, then conv."""
    k = w.shape[-1]
    h, wd = x.shape[-2:]
    ph = max((math.ceil(h / stride) - 1) * stride + k - h, 0)
    pw = max((math.ceil(wd / stride) - 1) * stride + k - wd, 0)
    x = F.pad(x, [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2])
    return F.conv2d(x, w, stride=stride, groups=groups)


@pytest.mark.parametrize("k,s,hw,c", [(3, 1, (9, 13), 24), (3, 2, (10, 12), 16), (5, 1, (7, 11), 8),
                                      (5, 2, (12, 17), 40), (5, 2, (15, 20), 12), (3, 2, (1, 1), 4),
                                      (5, 1, (30, 41), 264), (3, 1, (2, 3), 8), (5, 1, (1, 1), 4)])
def test_dwconv_same(mf, k, s, hw, c):
    x, w = rnd(2, c, *hw, seed=1), rnd(c, 1, k, k, seed=2, scale=0.5)
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = tf_same_ref(xr, wr, s, c)
    dy = rnd(*yr.shape, seed=3)
    yr.backward(dy)
    xg = nhwc(x).float().to(DEV).requires_grad_()
    wg = w.float().to(DEV).requires_grad_()
    yg = mf.dwconv_nhwc(xg, wg, stride=s)
    yg.backward(nhwc(dy).float().to(DEV))
    close(nchw(yg), yr)
    close(nchw(xg.grad), xr.grad)
    n_acc = 2 * yr.shape[-1] * yr.shape[-2]
    close(wg.grad, wr.grad, rtol=1e-5 * math.sqrt(n_acc))


@pytest.mark.parametrize("n,c,r,h,w", [(3, 48, 12, 7, 9), (2, 600, 26, 5, 6), (2, 3072, 128, 2, 3)])
def test_squeeze_excite(mf, n, c, r, h, w):
    x, wr, br = rnd(n, c, h, w, seed=4, scale=2), rnd(r, c, seed=5, scale=0.3), rnd(r, seed=6)
    we, be = rnd(c, r, seed=7, scale=0.3), rnd(c, seed=8)
    ts = [t.clone().requires_grad_() for t in (x, wr, br, we, be)]
    xs = ts[0].mean((2, 3))
    z = F.silu(xs @ ts[1].T + ts[2])
    yr = ts[0] * torch.sigmoid(z @ ts[3].T + ts[4])[:, :, None, None]
    dy = rnd(*yr.shape, seed=9)
    yr.backward(dy)
    gs = [nhwc(x).float().to(DEV)] + [t.float().to(DEV) for t in (wr, br, we, be)]
    gs = [t.requires_grad_() for t in gs]
    yg = mf.squeeze_excite(*gs)
    yg.backward(nhwc(dy).float().to(DEV))
    close(nchw(yg), yr)
    close(nchw(gs[0].grad), ts[0].grad)
    for a, b in zip(gs[1:], ts[1:]):
        close(a.grad, b.grad, rtol=1e-4)


def test_spatial_mean(mf):
    x = rnd(2, 256, 64, seed=10)
    xr = x.clone().requires_grad_()
    yr = xr.mean(1)
    dy = rnd(2, 64, seed=11)
    yr.backward(dy)
    xg = x.float().to(DEV).requires_grad_()
    yg = mf.spatial_mean(xg)
    yg.backward(dy.float().to(DEV))
    close(yg, yr)
    close(xg.grad, xr.grad)


@pytest.mark.parametrize("rows,cols,scale", [(37, 300, 0.18), (5, 19200, 0.125), (64, 256, 1.0), (3, 6, 0.5),
                                             (2, 1025, 1.0)])
def test_softmax(mf, rows, cols, scale):
    x = rnd(rows, cols, seed=12, scale=4)
    xr = x.clone().requires_grad_()
    yr = torch.softmax(scale * xr, -1)
    dy = rnd(rows, cols, seed=13)
    yr.backward(dy)
    xg = x.float().to(DEV).requires_grad_()
    yg = mf.softmax_lastdim(xg, scale)
    yg.backward(dy.float().to(DEV))
    close(yg, yr, rtol=1e-5)
    close(xg.grad, xr.grad, rtol=1e-4)


def test_dropout_mask_is_reproduced_in_backward(mf):
    torch.manual_seed(0)
    x = torch.ones(1 << 20, device=DEV).requires_grad_()
    y = mf.dropout(x, 0.1, True)
    keep = (y != 0)
    frac = keep.float().mean().item()
    assert abs(frac - 0.9) < 5e-3, frac
    assert torch.allclose(y[keep], torch.full_like(y[keep], 1 / 0.9))
    y.backward(torch.ones_like(y))
    assert torch.equal(x.grad != 0, keep)
    assert mf.dropout(x, 0.1, False) is x


def _uniform01_np(seed, ctr):
    """heads.hip uniform01: splitmix64 of seed + golden * (ctr + 1), top 24 bits."""
    import numpy as np
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * (ctr.astype(np.uint64) + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(40)).astype(np.float64) / 16777216.0


@pytest.mark.parametrize("n,shift", [(4096, 0), (4099, 0), (4096, 1)])
def test_dropout_dev_mask_matches_hash(mf, n, shift):
    """mdemi_dropout_dev: the float4 form (n % 4 == 0, aligned) and the scalar form draw the
    same mask, element for element, as the hash restated in numpy."""
    import numpy as np
    from mdemi import _lib as L
    base = torch.randn(n + shift, device=DEV)
    x = base[shift:]
    y = torch.empty_like(x)
    seed = torch.tensor([123456789], device=DEV, dtype=torch.int64)
    L.call("mdemi_dropout_dev", x.data_ptr(), y.data_ptr(), n, 0.3, seed.data_ptr(), 5, 1000, L.stream())
    torch.cuda.synchronize()
    u = _uniform01_np(123456789 + 5, np.arange(n, dtype=np.uint64) + np.uint64(1000))
    want = np.where(u >= np.float32(0.3), x.cpu().numpy() * np.float32(1 / 0.7), 0.0).astype(np.float32)
    got = y.cpu().numpy()
    assert np.array_equal(got != 0, want != 0)
    np.testing.assert_allclose(got, want, rtol=1e-6)


@pytest.mark.parametrize("B,H,W,K", [(2, 5, 7, 256), (1, 3, 4, 32), (3, 16, 20, 128), (2, 48, 64, 256),
                                     (1, 17, 23, 64), (2, 9, 31, 512), (1, 6, 6, 36)])
def test_bin_head_nhwc(mf, B, H, W, K):
    lg, c = rnd(B, K, H, W, seed=14, scale=3), rnd(B, K, seed=15, scale=5).abs()
    lr, cr = lg.clone().requires_grad_(), c.clone().requires_grad_()
    pr = (torch.softmax(lr, 1) * cr[:, :, None, None]).sum(1, keepdim=True)
    dy = rnd(*pr.shape, seed=16)
    pr.backward(dy)
    lgg, cg = nhwc(lg).float().to(DEV).requires_grad_(), c.float().to(DEV).requires_grad_()
    pg = mf.bin_head_nhwc(lgg, cg)
    pg.backward(dy.float().to(DEV))
    close(pg, pr)
    close(nchw(lgg.grad), lr.grad)
    close(cg.grad, cr.grad, rtol=1e-5 * math.sqrt(H * W))


@pytest.mark.parametrize("mode", [0, 1])
def test_bins(mf, mode):
    B, K, lo, hi = 3, 256, 1e-3, 10.0
    raw = rnd(B, K, seed=17, scale=2)
    rr = raw.clone().requires_grad_()
    w = (F.relu(rr) + 0.1) if mode == 0 else (F.elu(rr, alpha=0.1) + 0.1)
    w = w / w.sum(1, keepdim=True)
    e = torch.cumsum(F.pad((hi - lo) * w, (1, 0), value=lo), 1)
    cen = 0.5 * (e[:, :-1] + e[:, 1:])
    dc, de = rnd(B, K, seed=18), rnd(B, K + 1, seed=19)
    ((cen * dc).sum() + (e * de).sum()).backward()
    rg = raw.float().to(DEV).requires_grad_()
    eg, cg = mf.bins_from_raw(rg, mode, lo, hi)
    ((cg * dc.float().to(DEV)).sum() + (eg * de.float().to(DEV)).sum()).backward()
    close(eg, e, rtol=1e-5)
    close(cg, cen, rtol=1e-5)
    close(rg.grad, rr.grad, rtol=1e-4)


def test_conv_replicate_pad(mf):
    """ConvBN's conv (layer_utils.py:18-22): 3x3, padding_mode='replicate', no bias."""
    x, w = rnd(2, 20, 7, 9, seed=20), rnd(12, 20, 3, 3, seed=21, scale=0.2)
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = F.conv2d(F.pad(xr, (1, 1, 1, 1), mode="replicate"), wr)
    dy = rnd(*yr.shape, seed=22)
    yr.backward(dy)
    from mdemi import _lib as L
    xg, wg = nhwc(x).float().to(DEV).requires_grad_(), w.float().to(DEV).requires_grad_()
    yg = mf.conv2d_nhwc(xg, wg, None, stride=1, pad=1, pad_mode=L.PAD_REPLICATE)
    yg.backward(nhwc(dy).float().to(DEV))
    close(nchw(yg), yr, rtol=1e-4)
    close(nchw(xg.grad), xr.grad, rtol=1e-4)
    close(wg.grad, wr.grad, rtol=1e-4)


def test_conv_1x1_padding_1(mf):
    """DecoderBN.conv2 (unet_adaptive_bins.py:32): 1x1 conv with padding=1 (border = bias)."""
    x, w, b = rnd(2, 8, 5, 6, seed=23), rnd(12, 8, 1, 1, seed=24), rnd(12, seed=25)
    xr, wr, br = [t.clone().requires_grad_() for t in (x, w, b)]
    yr = F.conv2d(xr, wr, br, padding=1)
    dy = rnd(*yr.shape, seed=26)
    yr.backward(dy)
    xg, wg, bg = nhwc(x).float().to(DEV).requires_grad_(), w.float().to(DEV).requires_grad_(), \
        b.float().to(DEV).requires_grad_()
    yg = mf.conv2d_nhwc(xg, wg, bg, stride=1, pad=1)
    yg.backward(nhwc(dy).float().to(DEV))
    close(nchw(yg), yr)
    close(nchw(xg.grad), xr.grad)
    close(wg.grad, wr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)


def test_stem_conv_same_stride2(mf):
    """EfficientNet conv_stem: 3x3 stride 2 TF-'same' on the image (channels padded to 4)."""
    x, w = rnd(2, 3, 16, 22, seed=27), rnd(8, 3, 3, 3, seed=28)
    yr = tf_same_ref(x, w, 2, 1)
    xg = mf.nchw_to_nhwc_pad(x.float().to(DEV), 4)
    w4 = F.pad(w, (0, 0, 0, 0, 0, 1)).float().to(DEV)
    oh, pt = mf.same_pad(16, 3, 2)
    ow, pl = mf.same_pad(22, 3, 2)
    assert pt == pl == 0
    yg = mf.conv2d_nhwc(xg, w4, None, stride=2, pad=0, out_hw=(oh, ow))
    close(nchw(yg), yr)


@pytest.mark.parametrize("B,Sq,Sk,heads,dqk,dv,p", [(2, 30, 30, 4, 8, 8, 0.0), (2, 16, 40, 1, 16, 16, 0.0),
                                                     (1, 40, 12, 2, 32, 32, 0.0), (2, 9, 9, 2, 4, 4, 0.3)])
def test_attention(mf, B, Sq, Sk, heads, dqk, dv, p):
    """q from one buffer, k and v as column slices of a shared buffer (fused projection)."""
    q = rnd(B * Sq, heads * dqk + 4, seed=30)
    kv = rnd(B * Sk, heads * (dqk + dv), seed=31)
    scale = dqk ** -0.5
    mask = None
    if p > 0:
        # the dropout mask is a hash of (seed, index): with the same torch seed, a run whose V_h is the
        # identity returns dropout(P) itself, which exposes the mask the real run uses
        eye = torch.eye(Sk).repeat(B, heads).float().to(DEV)
        torch.manual_seed(5)
        pd, _ = mf.attention(q.float().to(DEV), kv.float().to(DEV), eye, B, Sq, Sk, heads, dqk, Sk, scale, q_off=4,
                             k_off=0, v_off=0, p=p, training=True)
        mask = (pd.view(B, Sq, heads, Sk).transpose(1, 2) != 0).double().cpu()
        assert 0.6 < mask.mean().item() < 0.8
    qg = q.float().to(DEV).requires_grad_()
    kvg = kv.float().to(DEV).requires_grad_()
    torch.manual_seed(5)
    out, P = mf.attention(qg, kvg, kvg, B, Sq, Sk, heads, dqk, dv, scale, q_off=4, k_off=0, v_off=heads * dqk,
                          p=p, training=True)
    dy = rnd(B * Sq, heads * dv, seed=32)
    dP = rnd(B, heads, Sq, Sk, seed=33)
    ((out * dy.float().to(DEV)).sum() + (P * dP.float().to(DEV)).sum()).backward()
    qr, kvr = q.clone().requires_grad_(), kv.clone().requires_grad_()
    Q = qr[:, 4:].view(B, Sq, heads, dqk).transpose(1, 2)
    Kt = kvr[:, :heads * dqk].view(B, Sk, heads, dqk).transpose(1, 2)
    V = kvr[:, heads * dqk:].view(B, Sk, heads, dv).transpose(1, 2)
    Pr = torch.softmax(scale * Q @ Kt.transpose(-1, -2), -1)
    Pdr = Pr if mask is None else Pr * mask / (1 - p)
    Or = (Pdr @ V).transpose(1, 2).reshape(B * Sq, heads * dv)
    ((Or * dy).sum() + (Pr * dP).sum()).backward()
    close(P, Pr, rtol=1e-5)
    close(out, Or, rtol=1e-5)
    close(qg.grad, qr.grad, rtol=1e-4)
    close(kvg.grad, kvr.grad, rtol=1e-4)


def test_channel_norm_silu(mf):
    x, g, b = rnd(2, 16, 5, 7, seed=34, scale=2), rnd(16, seed=35), rnd(16, seed=36)
    xr, gr, br = [t.clone().requires_grad_() for t in (x, g, b)]
    yr = F.silu(F.batch_norm(xr, None, None, gr, br, training=True, eps=1e-3))
    dy = rnd(*yr.shape, seed=37)
    yr.backward(dy)
    from mdemi import _lib as L
    xg, gg, bg = nhwc(x).float().to(DEV).requires_grad_(), g.float().to(DEV).requires_grad_(), \
        b.float().to(DEV).requires_grad_()
    yg, _, _ = mf.batch_norm_nhwc(xg, gg, bg, 1e-3, L.ACT_SILU)
    yg.backward(nhwc(dy).float().to(DEV))
    close(nchw(yg), yr, rtol=1e-5)
    close(nchw(xg.grad), xr.grad, rtol=1e-4)
    close(gg.grad, gr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)


@pytest.mark.parametrize("n,c,h,w", [(2, 16, 5, 7), (3, 240, 30, 41), (8, 1824, 15, 20), (2, 48, 1, 1)])
def test_bn_train_pooled_for_squeeze_excite(mf, n, c, h, w):
    """mdemi_bn_train_fwd_pooled (BatchNormAct2d -> SqueezeExcite in the EfficientNet blocks):
    y, the statistics and the running update equal the plain training forward's bit for bit, and
    the per-image spatial mean it records equals y's mean in fp64 (to fp32 summation)."""
    from mdemi import _lib as L
    x, g, b = rnd(n, c, h, w, seed=70, scale=2), rnd(c, seed=71), rnd(c, seed=72)
    xg = nhwc(x).float().to(DEV)
    outs = []
    for pool in (False, True):
        rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
        nb = torch.zeros((), dtype=torch.int64, device=DEV)
        y, mean, rstd = mf.batch_norm_nhwc(xg, g.float().to(DEV), b.float().to(DEV), 1e-3, L.ACT_SILU,
                                           running=(rm, rv, nb, 0.1), pool=pool)
        outs.append((y, mean, rstd, rm, rv, nb, mf.pooled_of(y)))
    (y0, m0, r0, rm0, rv0, nb0, p0), (y1, m1, r1, rm1, rv1, nb1, p1) = outs
    assert p0 is None and p1 is not None
    for a, b_ in ((y0, y1), (m0, m1), (r0, r1), (rm0, rm1), (rv0, rv1), (nb0, nb1)):
        assert torch.equal(a, b_)
    ref = y1.double().mean(dim=(1, 2))
    close(p1, ref, rtol=1e-6, atol=1e-7)
    y1.add_(1.0)  # an in-place change invalidates the recorded mean
    assert mf.pooled_of(y1) is None


@pytest.mark.parametrize("act", ["silu", "relu"])
def test_mlp_act(mf, act):
    from mdemi import _lib as L
    M, C, Hd = 300, 64, 256
    x, w1, b1, w2, b2 = rnd(M, C, seed=38), rnd(Hd, C, seed=39, scale=0.2), rnd(Hd, seed=40), \
        rnd(C, Hd, seed=41, scale=0.1), rnd(C, seed=42)
    ts = [t.clone().requires_grad_() for t in (x, w1, b1, w2, b2)]
    f = F.silu if act == "silu" else F.relu
    yr = F.linear(f(F.linear(ts[0], ts[1], ts[2])), ts[3], ts[4]) + ts[0]
    dy = rnd(M, C, seed=43)
    yr.backward(dy)
    gs = [t.float().to(DEV).requires_grad_() for t in (x, w1, b1, w2, b2)]
    yg = mf.mlp(*gs, residual=gs[0], act=L.ACT_SILU if act == "silu" else L.ACT_RELU)
    yg.backward(dy.float().to(DEV))
    close(yg, yr, rtol=1e-4)
    for a, b in zip(gs, ts):
        close(a.grad, b.grad, rtol=1e-4)


def test_depth_metrics_match_reference_golden(mf):
    """utils/depth_utils.py metrics on the GPU vs the reference's own outputs (golden fixture)."""
    from golden_util import GOLDEN
    import os
    d = np.load(os.path.join(GOLDEN, "depth_metrics.npz"))
    gt, pred = d["in/gt"], d["in/pred"]
    H, W = gt.shape
    from mdemi.utils.depth_utils import eval_crop_rect
    names = ["a1", "a2", "a3", "abs_rel", "sq_rel", "rmse", "rmse_log", "silog", "log_10"]
    for case, eo, dt in [("nyu_eigen", {"garg_crop": False, "eigen_crop": True}, "NYU"),
                         ("kitti_garg", {"garg_crop": True, "eigen_crop": False}, "KITTI"),
                         ("kitti_eigen", {"garg_crop": False, "eigen_crop": True}, "KITTI")]:
        rect = eval_crop_rect(eo, H, W, dt)
        out = mf.depth_metrics(torch.from_numpy(pred)[None, None].to(DEV), torch.from_numpy(gt)[None, None].to(DEV),
                               rect, 0.0, 1e9, clamp_pred=False).cpu().numpy()[0]
        assert int(out[9]) == int(d[f"mask/{case}"].sum())
        for i, nme in enumerate(names):
            ref = float(d[f"err/{case}/{nme}"])
            assert abs(out[i] - ref) <= 2e-6 * abs(ref) + 1e-9, (case, nme, out[i], ref)


def test_patch_conv_dgrad(mf):
    """stride == kernel conv (mViT embedding_encoder, layers.py:13-18): input gradient by column
    GEMM + NHWC scatter; rows/cols dropped by the floor get zero."""
    x, w, b = rnd(2, 8, 13, 17, seed=50), rnd(12, 8, 4, 4, seed=51, scale=0.3), rnd(12, seed=52)
    xr, wr, br = [t.clone().requires_grad_() for t in (x, w, b)]
    yr = F.conv2d(xr, wr, br, stride=4)
    dy = rnd(*yr.shape, seed=53)
    yr.backward(dy)
    xg, wg, bg = nhwc(x).float().to(DEV).requires_grad_(), w.float().to(DEV).requires_grad_(), \
        b.float().to(DEV).requires_grad_()
    yg = mf.conv2d_nhwc(xg, wg, bg, stride=4, pad=0)
    yg.backward(nhwc(dy).float().to(DEV))
    close(nchw(yg), yr, rtol=1e-4)
    close(nchw(xg.grad), xr.grad, rtol=1e-4)
    close(wg.grad, wr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)


@pytest.mark.parametrize("shape", [(2, 3, 5, 16), (1, 1, 7, 13), (3, 2, 4, 1), (2, 3, 480, 640)])
def test_flip_w_and_flip_avg(mf, shape):
    """Flip-eval sweeps (eval.flip_eval): bit-exact flip, (a + flip(b)) / 2 in fp32; both the
    float4 path (W % 4 == 0) and the scalar path, and an unaligned view."""
    a, b = rnd(*shape, seed=60).float(), rnd(*shape, seed=61).float()
    ag, bg = a.to(DEV), b.to(DEV)
    assert torch.equal(mf.flip_w(ag).cpu(), torch.flip(a, dims=[-1]))
    want = (a + torch.flip(b, dims=[-1])) * 0.5
    assert torch.equal(mf.flip_avg_w(ag, bg).cpu(), want)
    # storage offset of one float: the kernel must take the scalar path
    buf = torch.zeros(a.numel() + 1, device=DEV)
    buf[1:] = ag.reshape(-1)
    av = buf[1:].view(shape)
    assert torch.equal(mf.flip_w(av).cpu(), torch.flip(a, dims=[-1]))
    assert torch.equal(mf.flip_avg_w(av, bg).cpu(), want)


@pytest.mark.parametrize("B,P,H,W", [(2, 16, 9, 13), (3, 256, 40, 70), (1, 7, 1, 1500)])
def test_bins_chamfer_loss_fwd_bwd(mf, B, P, H, W):
    """AdaBins chamfer loss (loss.chamfer_weight) vs the fp64 oracle restatement, loss and edge
    gradients; invalid (< 1e-3) GT pixels, several 1024-pixel chunks, ragged last chunk."""
    from oracle.adabins import bins_chamfer_loss
    g = torch.Generator().manual_seed(70 + P)
    widths = torch.rand(B, P, generator=g, dtype=torch.float64) + 0.1
    edges = torch.cat([torch.zeros(B, 1, dtype=torch.float64), widths.cumsum(1)], 1)
    edges = 1e-3 + edges / edges[:, -1:] * (10.0 - 1e-3)
    gt = torch.rand(B, 1, H, W, generator=g, dtype=torch.float64) * 9.5 + 0.5
    gt[torch.rand(B, 1, H, W, generator=g) < 0.3] = 0.0
    er = edges.clone().requires_grad_()
    ref = bins_chamfer_loss(er, gt)
    ref.backward()
    eg = edges.float().to(DEV).requires_grad_()
    got = mf.bins_chamfer(eg, gt.float().to(DEV))
    got.backward(torch.tensor(1.7, device=DEV))
    close(got, ref.detach(), rtol=1e-5, atol=1e-7)
    close(eg.grad, 1.7 * er.grad, rtol=1e-4, atol=1e-7)


def test_bins_chamfer_loss_from_centres(mf):
    """Depthformer v8 form: centres (B, P, 1, 1) given directly (the oracle's chamfer, restated on
    centres)."""
    g = torch.Generator().manual_seed(77)
    B, P = 2, 32
    cen = torch.sort(torch.rand(B, P, generator=g, dtype=torch.float64) * 10, dim=1).values
    gt = torch.rand(B, 1, 30, 50, generator=g, dtype=torch.float64) * 9.5 + 0.5
    gt[:, :, :5] = 0.0
    cr = cen.clone().requires_grad_()
    d_ref = 0.0
    for c, t in zip(cr, gt.flatten(1)):
        t = t[t >= 1e-3]
        d = (c[:, None] - t[None, :]) ** 2
        d_ref = d_ref + d.min(1).values.mean() + d.min(0).values.mean()
    d_ref = d_ref / B
    d_ref.backward()
    cg = cen.float().to(DEV).view(B, P, 1, 1).requires_grad_()
    got = mf.bins_chamfer(cg, gt.float().to(DEV), from_edges=False)
    got.backward()
    close(got, d_ref.detach(), rtol=1e-5, atol=1e-7)
    close(cg.grad.view(B, P), cr.grad, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_gemm_two_level_batch(mf, prec):
    """batch_inner: entry z = o * n + i reads A at o*sa + i*sa2, B at o*sb + i*sb2 and writes C at
    o*sc + i*sc2 -- per-head column slices of token-major buffers, as the attention op uses."""
    from mdemi import _lib as L
    Bo, n, M, N, K = 3, 4, 37, 24, 20
    A = rnd(Bo * M, n * K + 4, seed=60).float().to(DEV)        # [B*M, heads*K (+4 unused)]
    Bm = rnd(Bo * N, n * K, seed=61).float().to(DEV)           # [B*N, heads*K]
    C = torch.full((Bo, n, M, N), float("nan"), device=DEV)
    with mf.matmul_precision(prec):
        mf.gemm(A, Bm, C, M, N, K, lda=n * K + 4, ldb=n * K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
                batch=Bo * n, a_bstride=M * (n * K + 4), b_bstride=N * n * K, c_bstride=n * M * N, a_off=4,
                inner=(n, K, K, M * N))
    torch.cuda.synchronize()
    Ar = A[:, 4:].double().cpu().view(Bo, M, n, K).transpose(1, 2)
    Br = Bm.double().cpu().view(Bo, N, n, K).transpose(1, 2)
    ref = Ar @ Br.transpose(-1, -2)
    tol = 1e-5 if prec == "fp32" else 2e-2
    assert torch.isfinite(C).all()
    close(C, ref, rtol=tol)


@pytest.mark.parametrize("kind", ["kk", "kmn", "mnmn_rowsum", "conv"])
def test_gemm_f32_variants_bit_identical(mf, kind):
    """Every fp32 pipelining variant (incl. the 256-row tiles 6 and 7, which the autotuner may
    pick per shape) adds each output's products in the same order: results are bit-identical,
    so the tuner's choice never changes a number.  Shapes straddle tile edges (M = 300)."""
    from mdemi import _lib as L
    lib = L.load()
    M, N, K = 300, 136, 200
    outs = []
    for v in range(8):
        lib.mdemi_gemm_set_variant(v, 8)
        try:
            if kind == "kk":
                A, B = rnd(M, K, seed=70).float().to(DEV), rnd(N, K, seed=71).float().to(DEV)
                C = torch.empty(M, N, device=DEV)
                mf.gemm(A, B, C, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, split_k=1)
                outs.append((C.clone(),))
            elif kind == "kmn":
                A, B = rnd(M, K, seed=72).float().to(DEV), rnd(K, N, seed=73).float().to(DEV)
                C = torch.empty(M, N, device=DEV)
                mf.gemm(A, B, C, M, N, K, lda=K, ldb=N, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG, split_k=3)
                outs.append((C.clone(),))
            elif kind == "mnmn_rowsum":  # weight-gradient form with the fused bias-gradient row sums
                A, B = rnd(K * 8, M, seed=74).float().to(DEV), rnd(K * 8, N, seed=75).float().to(DEV)
                C, rs = torch.empty(M, N, device=DEV), torch.empty(M, device=DEV)
                mf.gemm(A, B, C, M, N, K * 8, lda=M, ldb=N, ldc=N, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
                        rowsum_a=rs)
                outs.append((C.clone(), rs.clone()))
            else:
                x = rnd(2, 13, 17, 20, seed=76).float().to(DEV)
                w = rnd(24, 20, 3, 3, seed=77).float().to(DEV)
                outs.append((mf.conv2d_nhwc(x, w, None, stride=1, pad=1).clone(),))
            torch.cuda.synchronize()
        finally:
            lib.mdemi_gemm_set_variant(-1, 8)
    for v in range(1, 8):
        for a, b in zip(outs[0], outs[v]):
            assert torch.equal(a, b), (kind, v, (a - b).abs().max().item())
    if kind == "kk":
        close(outs[0][0], A.double().cpu() @ B.double().cpu().T, rtol=1e-5)
