"""Kernel-level numerics: every libmdemi kernel against a plain PyTorch fp64
CPU reference of the same op (forward and backward).  Tolerances are stated
per test; fp32 kernels are held to ~1e-5 relative on O(1) data."""
import math

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
    err = (a - b).abs().max().item()
    ref = b.abs().max().item()
    assert err <= atol + rtol * ref, f"max|diff|={err:.3e} max|ref|={ref:.3e}"


@pytest.fixture(scope="module")
def mf():
    from mdemi import functional as mf
    from mdemi import _lib
    _lib.load()
    return mf


@pytest.mark.parametrize("M,N,K", [(128, 128, 16), (300, 200, 70), (1, 5, 3), (517, 384, 192), (64, 1536, 384)])
def test_linear_fwd_bwd(mf, M, N, K):
    x, w, b = rnd(M, K, seed=1), rnd(N, K, seed=2, scale=0.1), rnd(N, seed=3)
    res = rnd(M, N, seed=4)
    dy = rnd(M, N, seed=5)
    xr, wr, br, rr = [t.clone().requires_grad_() for t in (x, w, b, res)]
    yr = F.linear(xr, wr, br) + rr
    yr.backward(dy)
    xg, wg, bg, rg = [t.float().to(DEV).requires_grad_() for t in (x, w, b, res)]
    yg = mf.linear(xg, wg, bg, residual=rg)
    yg.backward(dy.float().to(DEV))
    tol = dict(rtol=1e-5 * max(1, math.sqrt(K)), atol=1e-5)
    close(yg, yr, **tol)
    close(xg.grad, xr.grad, rtol=1e-5 * math.sqrt(N), atol=1e-5)
    close(wg.grad, wr.grad, rtol=1e-5 * math.sqrt(M), atol=1e-5)
    close(bg.grad, br.grad, rtol=1e-5 * math.sqrt(M), atol=1e-5)
    close(rg.grad, rr.grad)


def test_linear_gelu_on_load(mf):
    M, K, N = 333, 96, 48
    h, w, b = rnd(M, K, seed=6, scale=3), rnd(N, K, seed=7, scale=0.2), rnd(N, seed=8)
    dy = rnd(M, N, seed=9)
    hr, wr, br = [t.clone().requires_grad_() for t in (h, w, b)]
    yr = F.linear(F.gelu(hr), wr, br)
    yr.backward(dy)
    hg, wg, bg = [t.float().to(DEV).requires_grad_() for t in (h, w, b)]
    yg = mf.linear(hg, wg, bg, in_gelu=True)
    yg.backward(dy.float().to(DEV))
    close(yg, yr, rtol=1e-4)
    close(hg.grad, hr.grad, rtol=1e-4)
    close(wg.grad, wr.grad, rtol=1e-4)


@pytest.mark.parametrize("M,C", [(333, 24), (4100, 96)])
def test_mlp_fused(mf, M, C):
    """fc1 -> GELU -> fc2 + residual with fc1 writing both h and gelu(h)."""
    x, w1, b1 = rnd(M, C, seed=20), rnd(4 * C, C, seed=21, scale=0.3), rnd(4 * C, seed=22)
    w2, b2, res = rnd(C, 4 * C, seed=23, scale=0.2), rnd(C, seed=24), rnd(M, C, seed=25)
    dy = rnd(M, C, seed=26)
    ref = [t.clone().requires_grad_() for t in (x, w1, b1, w2, b2, res)]
    yr = F.linear(F.gelu(F.linear(ref[0], ref[1], ref[2])), ref[3], ref[4]) + ref[5]
    yr.backward(dy)
    gpu = [t.float().to(DEV).requires_grad_() for t in (x, w1, b1, w2, b2, res)]
    yg = mf.mlp(*gpu)
    yg.backward(dy.float().to(DEV))
    close(yg, yr, rtol=1e-4)
    for a, b in zip(gpu, ref):
        close(a.grad, b.grad, rtol=1e-4 * max(1, math.sqrt(M / 300)))


def test_gemm_splitk_and_batch(mf):
    from mdemi import _lib as L
    B, M, N, K = 3, 70, 90, 1000
    a, b = rnd(B, M, K, seed=10), rnd(B, N, K, seed=11)
    ref = torch.einsum("bmk,bnk->bmn", a, b)
    ag, bg = a.float().to(DEV), b.float().to(DEV)
    for split in (1, 7):
        c = torch.empty(B, M, N, device=DEV)
        mf.gemm(ag, bg, c, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, batch=B,
                a_bstride=M * K, b_bstride=N * K, c_bstride=M * N, split_k=split)
        close(c, ref, rtol=1e-4)


@pytest.mark.parametrize("cin,cout,k,s,p,hw", [(8, 16, 3, 1, 1, (9, 13)), (64, 32, 3, 1, 1, (15, 20)),
                                              (12, 8, 1, 1, 0, (7, 5)), (16, 24, 3, 2, 1, (11, 10))])
def test_conv2d_nhwc(mf, cin, cout, k, s, p, hw):
    n = 2
    x, w, b = rnd(n, cin, *hw, seed=12), rnd(cout, cin, k, k, seed=13, scale=0.2), rnd(cout, seed=14)
    xr, wr, br = [t.clone().requires_grad_() for t in (x, w, b)]
    yr = F.conv2d(xr, wr, br, stride=s, padding=p)
    dy = rnd(*yr.shape, seed=15)
    yr.backward(dy)
    xg = x.permute(0, 2, 3, 1).contiguous().float().to(DEV).requires_grad_()
    wg, bg = w.float().to(DEV).requires_grad_(), b.float().to(DEV).requires_grad_()
    yg = mf.conv2d_nhwc(xg, wg, bg, stride=s, pad=p)
    close(yg.permute(0, 3, 1, 2), yr, rtol=1e-4)
    need_dx = s == 1
    if not need_dx:
        xg = xg.detach()
        yg = mf.conv2d_nhwc(xg, wg, bg, stride=s, pad=p)
    yg.backward(dy.permute(0, 2, 3, 1).float().to(DEV))
    if need_dx:
        close(xg.grad.permute(0, 3, 1, 2), xr.grad, rtol=1e-4)
    close(wg.grad, wr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)


@pytest.mark.parametrize("rows,C", [(1000, 192), (37, 1536), (5, 3072), (100, 64)])
def test_layernorm(mf, rows, C):
    x, g, b = rnd(rows, C, seed=16, scale=2) + 0.5, rnd(C, seed=17), rnd(C, seed=18)
    dy = rnd(rows, C, seed=19)
    xr, gr, br = [t.clone().requires_grad_() for t in (x, g, b)]
    yr = F.layer_norm(xr, (C,), gr, br, 1e-5)
    yr.backward(dy)
    xg, gg, bg = [t.float().to(DEV).requires_grad_() for t in (x, g, b)]
    yg = mf.layer_norm(xg, gg, bg, 1e-5)
    yg.backward(dy.float().to(DEV))
    close(yg, yr, rtol=1e-5)
    close(xg.grad, xr.grad, rtol=1e-4)
    close(gg.grad, gr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)


def _ref_window_attn(qk, qk_bias, v, v_bias, rpb, B, H, W, heads, ws, shift, scale, C, v_off):
    """Direct restatement of WindowAttention + pad/roll/partition (swin_transformer.py:112-240)."""
    hd = C // heads
    rows = B * H * W
    q = qk[:, :C]
    k = qk[:, C:2 * C]
    vv = v[:, v_off:v_off + C]
    Hp, Wp = -(-H // ws) * ws, -(-W // ws) * ws

    def grid(t, pad):
        t = t.view(B, H, W, C)
        full = (pad.view(1, 1, 1, C) if pad is not None else torch.zeros(1, 1, 1, C, dtype=t.dtype)).expand(
            B, Hp, Wp, C).clone()
        full[:, :H, :W] = t
        if shift:
            full = torch.roll(full, (-shift, -shift), (1, 2))
        return full.view(B, Hp // ws, ws, Wp // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, C)

    qw = grid(q, qk_bias[:C] if qk_bias is not None else None)
    kw = grid(k, qk_bias[C:2 * C] if qk_bias is not None else None)
    vw = grid(vv, v_bias[v_off:v_off + C] if v_bias is not None else None)
    nW = qw.shape[0] // B
    qh = qw.view(-1, ws * ws, heads, hd).transpose(1, 2) * scale
    kh = kw.view(-1, ws * ws, heads, hd).transpose(1, 2)
    vh = vw.view(-1, ws * ws, heads, hd).transpose(1, 2)
    attn = qh @ kh.transpose(-2, -1)
    coords = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")).flatten(1)
    rel = (coords[:, :, None] - coords[:, None, :]).permute(1, 2, 0)
    idx = (rel[..., 0] + ws - 1) * (2 * ws - 1) + rel[..., 1] + ws - 1
    attn = attn + rpb[idx.view(-1)].view(ws * ws, ws * ws, heads).permute(2, 0, 1).unsqueeze(0)
    if shift:
        img = torch.zeros(1, Hp, Wp, 1, dtype=qk.dtype)
        cnt = 0
        for hs in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            for wsl in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
                img[:, hs, wsl, :] = cnt
                cnt += 1
        mw = img.view(1, Hp // ws, ws, Wp // ws, ws, 1).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws)
        mask = mw.unsqueeze(1) - mw.unsqueeze(2)
        mask = mask.masked_fill(mask != 0, -100.0).masked_fill(mask == 0, 0.0)
        attn = attn.view(B, nW, heads, ws * ws, ws * ws) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, heads, ws * ws, ws * ws)
    attn = attn.softmax(-1)
    o = (attn @ vh).transpose(1, 2).reshape(-1, ws * ws, C)
    o = o.view(B, Hp // ws, Wp // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, Hp, Wp, C)
    if shift:
        o = torch.roll(o, (shift, shift), (1, 2))
    return o[:, :H, :W].reshape(rows, C)


@pytest.mark.parametrize("H,W,shift,swin", [(14, 14, 0, True), (10, 12, 3, True), (9, 16, 3, False),
                                            (7, 7, 3, True), (15, 20, 0, False)])
def test_window_attention(mf, H, W, shift, swin):
    B, heads, C, ws = 2, 2, 64, 7
    rows = B * H * W
    scale = (C // heads) ** -0.5
    rpb = rnd(169, heads, seed=20)
    if swin:
        qk = rnd(rows, 3 * C, seed=21)
        qkb = rnd(3 * C, seed=22)
        v, vb, v_off = qk, qkb, 2 * C
    else:
        qk = rnd(rows, 2 * C, seed=21)
        qkb = rnd(2 * C, seed=22)
        v, vb, v_off = rnd(rows, C, seed=23), None, 0
    dout = rnd(rows, C, seed=24)
    leaves = [qk, qkb, rpb] + ([] if swin else [v])
    refs = {id(t): t.clone().requires_grad_() for t in leaves}
    qk_r, qkb_r, rpb_r = refs[id(qk)], refs[id(qkb)], refs[id(rpb)]
    v_r = qk_r if swin else refs[id(v)]
    vb_r = qkb_r if swin else None
    out_r = _ref_window_attn(qk_r, qkb_r, v_r, vb_r, rpb_r, B, H, W, heads, ws, shift, scale, C, v_off)
    out_r.backward(dout)
    g = {k: t.detach().float().to(DEV).requires_grad_() for k, t in refs.items()}
    qk_g, qkb_g, rpb_g = g[id(qk)], g[id(qkb)], g[id(rpb)]
    v_g = qk_g if swin else g[id(v)]
    vb_g = qkb_g if swin else None
    out_g = mf.window_attention(qk_g, qkb_g, v_g, vb_g, rpb_g, B, H, W, heads, ws, shift, scale, C, v_off)
    out_g.backward(dout.float().to(DEV))
    close(out_g, out_r, rtol=1e-4)
    close(qk_g.grad, qk_r.grad, rtol=1e-4)
    close(qkb_g.grad, qkb_r.grad, rtol=1e-4)
    close(rpb_g.grad, rpb_r.grad, rtol=1e-4)
    if not swin:
        close(v_g.grad, v_r.grad, rtol=1e-4)


@pytest.mark.parametrize("B,K,H,W,softmax", [(2, 256, 24, 32, True), (3, 17, 5, 7, True), (2, 64, 8, 8, False)])
def test_bin_head(mf, B, K, H, W, softmax):
    logits = rnd(B, K, H, W, seed=30, scale=4)
    if not softmax:
        logits = logits.softmax(1)
    centers = rnd(B, K, seed=31).abs() * 10
    dpred = rnd(B, 1, H, W, seed=32)
    lr, cr = logits.clone().requires_grad_(), centers.clone().requires_grad_()
    pr = lr.softmax(1) if softmax else lr
    pred_r = (pr * cr.view(B, K, 1, 1)).sum(1, keepdim=True)
    pred_r.backward(dpred)
    lg, cg = logits.float().to(DEV).requires_grad_(), centers.float().to(DEV).requires_grad_()
    pred_g = mf.bin_head(lg, cg, do_softmax=softmax)
    pred_g.backward(dpred.float().to(DEV))
    close(pred_g, pred_r, rtol=1e-5)
    close(lg.grad, lr.grad, rtol=1e-4, atol=1e-5)
    close(cg.grad, cr.grad, rtol=1e-4)


@pytest.mark.parametrize("per_image,unbiased", [(False, False), (True, False), (True, True)])
def test_silog(mf, per_image, unbiased):
    B, H, W = 3, 40, 52
    gt = rnd(B, 1, H, W, seed=40).abs() * 9 + 0.5
    gt[:, :, :5] = 0.0  # invalid region
    pred = rnd(B, 1, H, W, seed=41).abs() * 9 + 0.5
    alpha, beta, md = 10.0, 0.15, 1e-3
    pr = pred.clone().requires_grad_()

    def group_loss(p, g):
        m = g > md
        d = torch.log(p[m]) - torch.log(g[m])
        var = d.var() if unbiased else (d * d).mean() - d.mean() ** 2
        return alpha * torch.sqrt(var + beta * d.mean() ** 2)

    if per_image:
        lr = torch.stack([group_loss(pr[b], gt[b]) for b in range(B)]).mean()
    else:
        lr = group_loss(pr, gt)
    lr.backward()
    pg = pred.float().to(DEV).requires_grad_()
    lg = mf.silog_loss(pg, gt.float().to(DEV), md, alpha, beta, per_image, unbiased)
    lg.backward()
    close(lg, lr, rtol=1e-5)
    close(pg.grad, pr.grad, rtol=1e-3, atol=1e-7)


@pytest.mark.parametrize("hw,out,align,sf", [((15, 20), (60, 80), False, 4.0), ((3, 3), (15, 20), False, None),
                                             ((30, 40), (60, 80), True, None), ((1, 1), (15, 20), False, None),
                                             ((7, 9), (5, 4), True, None)])
def test_bilinear(mf, hw, out, align, sf):
    n, c = 2, 8
    x = rnd(n, c, *hw, seed=50)
    xr = x.clone().requires_grad_()
    if sf is not None:
        yr = F.interpolate(xr, scale_factor=sf, mode="bilinear", align_corners=align)
    else:
        yr = F.interpolate(xr, size=out, mode="bilinear", align_corners=align)
    dy = rnd(*yr.shape, seed=51)
    yr.backward(dy)
    xg = x.permute(0, 2, 3, 1).contiguous().float().to(DEV).requires_grad_()
    yg = mf.interpolate_bilinear(xg, size=None if sf else out, scale_factor=sf, align_corners=align)
    yg.backward(dy.permute(0, 2, 3, 1).float().to(DEV))
    close(yg.permute(0, 3, 1, 2), yr)
    close(xg.grad.permute(0, 3, 1, 2), xr.grad, rtol=1e-5)


@pytest.mark.parametrize("is_bn,groups,act", [(True, 0, 2), (True, 0, 0), (False, 256, 2), (False, 4, 0)])
def test_channel_norm(mf, is_bn, groups, act):
    from mdemi import _lib as L
    n, c, h, w = 4, 512 if not is_bn else 48, 3, 5
    x = rnd(n, c, h, w, seed=60, scale=3) + 1
    g, b = rnd(c, seed=61), rnd(c, seed=62)
    dy = rnd(n, c, h, w, seed=63)
    xr, gr, br = [t.clone().requires_grad_() for t in (x, g, b)]
    if is_bn:
        yr = F.batch_norm(xr, None, None, gr, br, training=True, eps=1e-5)
    else:
        yr = F.group_norm(xr, groups, gr, br, eps=1e-5)
    if act == L.ACT_RELU:
        yr = F.relu(yr)
    yr.backward(dy)
    xg = x.permute(0, 2, 3, 1).contiguous().float().to(DEV).requires_grad_()
    gg, bg = g.float().to(DEV).requires_grad_(), b.float().to(DEV).requires_grad_()
    if is_bn:
        yg, _, _ = mf.batch_norm_nhwc(xg, gg, bg, 1e-5, act)
    else:
        yg = mf.group_norm_nhwc(xg, gg, bg, groups, 1e-5, act)
    yg.backward(dy.permute(0, 2, 3, 1).float().to(DEV))
    close(yg.permute(0, 3, 1, 2), yr, rtol=1e-5)
    close(xg.grad.permute(0, 3, 1, 2), xr.grad, rtol=1e-4)
    close(gg.grad, gr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)


@pytest.mark.parametrize("n,c,h,w,act", [(2, 48, 120, 160, 6), (2, 600, 9, 11, 3), (1, 1100, 7, 9, 0),
                                         (3, 6, 10, 10, 2), (4, 24, 1, 1, 6), (2, 2048, 15, 20, 3)])
def test_batch_norm_shapes(mf, n, c, h, w, act):
    """Training BatchNorm + fused activation over NHWC: the vectorised path (C % 4 == 0) with
    many row lanes per channel quad (C=48, 24), one lane with idle threads (C=600), several quad
    passes per block (C=1100, 2048), and the scalar path (C=6)."""
    from mdemi import _lib as L
    x = rnd(n, c, h, w, seed=64, scale=3) + 1
    g, b = rnd(c, seed=65), rnd(c, seed=66)
    dy = rnd(n, c, h, w, seed=67)
    xr, gr, br = [t.clone().requires_grad_() for t in (x, g, b)]
    yr = F.batch_norm(xr, None, None, gr, br, training=True, eps=1e-3)
    yr = {L.ACT_RELU: F.relu, L.ACT_SILU: F.silu, L.ACT_LEAKY: F.leaky_relu, L.ACT_NONE: lambda t: t}[act](yr)
    yr.backward(dy)
    xg = x.permute(0, 2, 3, 1).contiguous().float().to(DEV).requires_grad_()
    gg, bg = g.float().to(DEV).requires_grad_(), b.float().to(DEV).requires_grad_()
    yg, _, _ = mf.batch_norm_nhwc(xg, gg, bg, 1e-3, act)
    yg.backward(dy.permute(0, 2, 3, 1).float().to(DEV))
    close(yg.permute(0, 3, 1, 2), yr, rtol=1e-5)
    close(xg.grad.permute(0, 3, 1, 2), xr.grad, rtol=1e-4)
    close(gg.grad, gr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)


@pytest.mark.parametrize("momentum", [0.1, None])
def test_batch_norm_running_stats(mf, momentum):
    """bn_forward (the model-side BatchNorm2d) updates running_mean / running_var / the batch
    counter exactly as nn.BatchNorm2d does in training (unbiased variance, momentum or
    cumulative average), through mdemi_bn_running_update."""
    from mdemi.model.NewCRFs.uper_crf_head import bn_forward
    c = 40
    ref = torch.nn.BatchNorm2d(c, eps=1e-3, momentum=momentum).double()
    bn = torch.nn.BatchNorm2d(c, eps=1e-3, momentum=momentum).to(DEV)
    for step in range(3):
        x = rnd(2, c, 5, 7, seed=90 + step, scale=2) + 0.5
        ref(x)
        bn_forward(bn, x.permute(0, 2, 3, 1).contiguous().float().to(DEV))
    close(bn.running_mean, ref.running_mean, rtol=1e-5, atol=1e-6)
    close(bn.running_var, ref.running_var, rtol=1e-5, atol=1e-6)
    assert int(bn.num_batches_tracked) == 3


@pytest.mark.parametrize("n,c,h,w,act,affine_grad", [(2, 48, 30, 40, 6, True), (2, 600, 9, 11, 3, True),
                                                     (3, 6, 10, 10, 2, True), (2, 64, 7, 9, 0, False),
                                                     (1, 5, 4, 4, 6, False)])
def test_batch_norm_eval_backward(mf, n, c, h, w, act, affine_grad):
    """Eval-mode BatchNorm inside a training step (freeze_bn, common_utils.py:78-81): forward
    with the running statistics and gradients to the input and, unless frozen, the affine
    parameters -- F.batch_norm(training=False) in fp64, through mdemi_bn_frozen_bwd (vector
    path C % 4 == 0 and scalar path; dgamma/dbeta skipped when the affine is frozen)."""
    from mdemi import _lib as L
    x = rnd(n, c, h, w, seed=70, scale=3) + 1
    g, b = rnd(c, seed=71), rnd(c, seed=72)
    rm, rv = rnd(c, seed=73), rnd(c, seed=74).abs() + 0.5
    dy = rnd(n, c, h, w, seed=75)
    xr = x.clone().requires_grad_()
    gr, br = [t.clone().requires_grad_(affine_grad) for t in (g, b)]
    yr = F.batch_norm(xr, rm, rv, gr, br, training=False, eps=1e-3)
    yr = {L.ACT_RELU: F.relu, L.ACT_SILU: F.silu, L.ACT_LEAKY: F.leaky_relu, L.ACT_NONE: lambda t: t}[act](yr)
    yr.backward(dy)
    xg = x.permute(0, 2, 3, 1).contiguous().float().to(DEV).requires_grad_()
    gg, bg = [t.float().to(DEV).requires_grad_(affine_grad) for t in (g, b)]
    rmg, rvg = rm.float().to(DEV), rv.float().to(DEV)
    yg = mf.batch_norm_eval_nhwc(xg, gg, bg, rmg, rvg, 1e-3, act)
    yg.backward(dy.permute(0, 2, 3, 1).float().to(DEV))
    close(yg.permute(0, 3, 1, 2), yr, rtol=1e-5)
    close(xg.grad.permute(0, 3, 1, 2), xr.grad, rtol=1e-4)
    if affine_grad:
        close(gg.grad, gr.grad, rtol=1e-4)
        close(bg.grad, br.grad, rtol=1e-4)
    else:
        assert gg.grad is None and bg.grad is None
    close(rmg, rm, rtol=0)  # running statistics untouched in eval mode
    with torch.no_grad():  # no-grad path: one launch, same values
        close(mf.batch_norm_eval_nhwc(xg.detach(), gg, bg, rmg, rvg, 1e-3, act), yg.detach(), rtol=0)


def test_freeze_bn_train_step_reaches_encoder(mf):
    """A training step with every BatchNorm frozen (eval mode) still gives the parameters
    below each BN a gradient: AdaBins-style conv -> BN -> act stack, compared with torch."""
    from mdemi.model.NewCRFs.uper_crf_head import bn_forward
    from mdemi import _lib as L
    torch.manual_seed(3)
    conv = torch.nn.Conv2d(8, 16, 3, padding=1, bias=False).double()
    bn = torch.nn.BatchNorm2d(16, eps=1e-5).double()
    with torch.no_grad():
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
    bn.eval()
    x = rnd(2, 8, 12, 10, seed=76)
    F.relu(bn(conv(x))).sum().backward()
    w = conv.weight.detach().float().to(DEV).requires_grad_()
    bng = torch.nn.BatchNorm2d(16, eps=1e-5).to(DEV)
    bng.load_state_dict({k: v.float() for k, v in bn.state_dict().items()})
    bng.eval()
    xg = x.permute(0, 2, 3, 1).contiguous().float().to(DEV)
    yg = mf.conv2d_nhwc(xg, w, None, stride=1, pad=1)
    bn_forward(bng, yg, L.ACT_RELU).sum().backward()
    assert w.grad is not None and bng.weight.grad is not None
    close(w.grad, conv.weight.grad, rtol=1e-4)
    close(bng.weight.grad, bn.weight.grad, rtol=1e-4)
    assert int(bng.num_batches_tracked) == 0


@pytest.mark.parametrize("rows,C", [(300, 64), (1000, 192), (77, 1536)])
def test_layer_norm_skip(mf, rows, C):
    """(LN(x), x) residual pattern: z = x + LN(x) W^T; the skip gradient is summed inside the
    LayerNorm backward (mdemi_layernorm_bwd_add) -- value and all gradients vs fp64."""
    x, g, b = rnd(rows, C, seed=80, scale=2), rnd(C, seed=81) + 1, rnd(C, seed=82)
    w = rnd(C, C, seed=83, scale=0.1)
    dz = rnd(rows, C, seed=84)
    xr, gr, br = [t.clone().requires_grad_() for t in (x, g, b)]
    zr = xr + F.layer_norm(xr, (C,), gr, br, 1e-5) @ w.t()
    zr.backward(dz)
    xg, gg, bg = [t.float().to(DEV).requires_grad_() for t in (x, g, b)]
    y, skip = mf.layer_norm_skip(xg, gg, bg, 1e-5)
    zg = mf.linear(y, w.float().to(DEV), None, residual=skip)
    zg.backward(dz.float().to(DEV))
    close(zg, zr, rtol=1e-5)
    close(xg.grad, xr.grad, rtol=1e-4)
    close(gg.grad, gr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)


def test_pixel_shuffle_avgpool_patch(mf):
    n, c, h, w = 2, 16, 5, 7
    x = rnd(n, c, h, w, seed=70)
    xr = x.clone().requires_grad_()
    yr = F.pixel_shuffle(xr, 2)
    dy = rnd(*yr.shape, seed=71)
    yr.backward(dy)
    xg = x.permute(0, 2, 3, 1).contiguous().float().to(DEV).requires_grad_()
    yg = mf.pixel_shuffle_nhwc(xg, 2)
    yg.backward(dy.permute(0, 2, 3, 1).float().to(DEV))
    # a pure permutation: bit-exact against the fp32-rounded reference
    close(yg.permute(0, 3, 1, 2), yr.float(), rtol=0, atol=0)
    close(xg.grad.permute(0, 3, 1, 2), xr.grad.float(), rtol=0, atol=0)
    for s in (1, 2, 3, 6):
        x = rnd(n, 12, 11, 19, seed=72 + s)
        xr = x.clone().requires_grad_()
        yr = F.adaptive_avg_pool2d(xr, s)
        dy = rnd(*yr.shape, seed=80 + s)
        yr.backward(dy)
        xg = x.permute(0, 2, 3, 1).contiguous().float().to(DEV).requires_grad_()
        yg = mf.adaptive_avg_pool_nhwc(xg, s)
        yg.backward(dy.permute(0, 2, 3, 1).float().to(DEV))
        close(yg.permute(0, 3, 1, 2), yr, rtol=1e-5)
        close(xg.grad.permute(0, 3, 1, 2), xr.grad, rtol=1e-5)
    img = rnd(2, 3, 22, 30, seed=90)
    w, b = rnd(24, 3, 4, 4, seed=91), rnd(24, seed=92)
    wr, br = w.clone().requires_grad_(), b.clone().requires_grad_()
    yr = F.conv2d(F.pad(img, (0, 2, 0, 2)), wr, br, stride=4)
    dy = rnd(*yr.shape, seed=93)
    yr.backward(dy)
    wg, bg = w.float().to(DEV).requires_grad_(), b.float().to(DEV).requires_grad_()
    yg = mf.patch_embed(img.float().to(DEV), wg, bg)
    yg.backward(dy.permute(0, 2, 3, 1).float().to(DEV))
    close(yg.permute(0, 3, 1, 2), yr, rtol=1e-5)
    close(wg.grad, wr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)
    x = rnd(2, 6, 4, 5, seed=94).float().to(DEV)
    close(mf.nhwc_to_nchw(mf.nchw_to_nhwc(x)), x.cpu(), rtol=0, atol=0)
    close(mf.nchw_to_nhwc(x), x.cpu().permute(0, 2, 3, 1), rtol=0, atol=0)


def test_fused_adamw_with_clip_matches_torch(mf):
    from mdemi.train import FusedAdamW
    torch.manual_seed(0)
    shapes = [(300, 7), (5,), (70000,), (3, 4, 5)]
    ps = [torch.randn(*s, device=DEV) for s in shapes]
    pr = [p.clone().requires_grad_() for p in ps]
    pg = [p.clone().requires_grad_() for p in ps]
    ref = torch.optim.AdamW(pr, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.1)
    opt = FusedAdamW(pg, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.1, max_grad_norm=0.5)
    for it in range(3):
        grads = [torch.randn(*s, device=DEV) * (it + 1) for s in shapes]
        for p, g in zip(pr, grads):
            p.grad = g.clone()
        for p, g in zip(pg, grads):
            p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(pr, 0.5)
        ref.step()
        opt.step()
    for a, b in zip(pg, pr):
        close(a, b, rtol=1e-5, atol=1e-6)


def test_fused_adamw_per_parameter_steps_match_torch(mf):
    """A parameter whose gradient first appears at step 3 is bias-corrected as its own
    step 1 (torch's per-parameter state["step"]); resuming from torch's state_dict keeps
    those counts (optim.py FusedAdamW)."""
    from mdemi.train import FusedAdamW
    torch.manual_seed(1)
    shapes = [(64, 3), (9,), (1,)]
    ps = [torch.randn(*s, device=DEV) for s in shapes]
    pr = [p.clone().requires_grad_() for p in ps]
    pg = [p.clone().requires_grad_() for p in ps]
    ref = torch.optim.AdamW(pr, lr=1e-2, weight_decay=0.05)
    opt = FusedAdamW(pg, lr=1e-2, weight_decay=0.05)
    for it in range(5):
        live = [0, 1] if it < 2 else [0, 1, 2]  # parameter 2 gets gradients from step 3 on
        for i in range(3):
            g = torch.randn(*shapes[i], device=DEV) if i in live else None
            pr[i].grad = None if g is None else g.clone()
            pg[i].grad = None if g is None else g.clone()
        ref.step()
        opt.step()
    torch.cuda.synchronize()
    assert opt.steps == [5, 5, 3]
    for a, b in zip(pg, pr):
        close(a, b, rtol=1e-5, atol=1e-6)
    # resume a fresh optimizer from torch's state and take two more steps on both
    pq = [p.detach().clone().requires_grad_() for p in pg]
    opt2 = FusedAdamW(pq, lr=1e-2, weight_decay=0.05)
    opt2.load_state_dict(ref.state_dict())
    assert opt2.steps == [5, 5, 3]
    for it in range(2):
        for i in range(3):
            g = torch.randn(*shapes[i], device=DEV)
            pr[i].grad, pq[i].grad = g.clone(), g.clone()
        ref.step()
        opt2.step()
    for a, b in zip(pq, pr):
        close(a, b, rtol=1e-5, atol=1e-6)
    sd = opt2.state_dict()
    assert [int(sd["state"][i]["step"]) for i in range(3)] == [7, 7, 5]


def test_headconv(mf):
    n, c, h, w = 2, 128, 9, 11
    x, wt, b = rnd(n, c, h, w, seed=100), rnd(1, c, 3, 3, seed=101, scale=0.1), rnd(1, seed=102)
    xr, wr, br = [t.clone().requires_grad_() for t in (x, wt, b)]
    yr = F.conv2d(xr, wr, br, padding=1)
    dy = rnd(*yr.shape, seed=103)
    yr.backward(dy)
    xg = x.permute(0, 2, 3, 1).contiguous().float().to(DEV).requires_grad_()
    wg, bg = wt.float().to(DEV).requires_grad_(), b.float().to(DEV).requires_grad_()
    yg = mf.conv2d_nhwc(xg, wg, bg, stride=1, pad=1)
    yg.backward(dy.permute(0, 2, 3, 1).float().to(DEV))
    close(yg.permute(0, 3, 1, 2), yr, rtol=1e-5)
    close(xg.grad.permute(0, 3, 1, 2), xr.grad, rtol=1e-5)
    close(wg.grad, wr.grad, rtol=1e-4)
    close(bg.grad, br.grad, rtol=1e-4)


def test_space_to_depth_concat_droppath(mf):
    n, h, w, c = 2, 9, 13, 8
    x = rnd(n, h, w, c, seed=110)
    xr = x.clone().requires_grad_()
    xp = F.pad(xr, (0, 0, 0, w % 2, 0, h % 2))
    yr = torch.cat([xp[:, 0::2, 0::2], xp[:, 1::2, 0::2], xp[:, 0::2, 1::2], xp[:, 1::2, 1::2]], -1)
    dy = rnd(*yr.shape, seed=111)
    yr.backward(dy)
    xg = x.float().to(DEV).requires_grad_()
    yg = mf.space_to_depth2(xg)
    yg.backward(dy.float().to(DEV))
    close(yg, yr.float(), rtol=0, atol=0)
    close(xg.grad, xr.grad.float(), rtol=0, atol=0)
    a, b = rnd(4, 5, 8, seed=112).float().to(DEV), rnd(4, 5, 12, seed=113).float().to(DEV)
    cat = mf.concat_channels([a, b])
    close(cat, torch.cat([a, b], -1).cpu(), rtol=0, atol=0)
    res, br = rnd(4, 30, seed=114).float().to(DEV), rnd(4, 30, seed=115).float().to(DEV).requires_grad_()
    torch.manual_seed(0)
    y = mf.drop_path_add(res, br, 0.5, True)
    kept = (y - res).abs().sum(1) > 0
    exp = res + br.detach() * 2.0 * kept.float().unsqueeze(1)
    close(y, exp.cpu(), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("M,N,K", [(24, 40, 300000), (144, 24, 123457), (240, 40, 70000)])
def test_gemm_deep_split_skinny_wgrad(mf, M, N, K):
    """Weight gradient of a narrow 1x1 conv over many pixels (dW = dY^T X, db = dY^T 1): deep
    split-K (up to 512 slabs) combined by column sums, with the bias row-sum folded in."""
    from mdemi import _lib as L
    split = mf._split_for(M, N, K)
    assert split >= 32
    dy = torch.randn(K, M, device=DEV)
    x = torch.randn(K, N, device=DEV)
    dw = torch.empty(M, N, device=DEV)
    db = torch.empty(M, device=DEV)
    mf.gemm(dy, x, dw, M, N, K, lda=M, ldb=N, ldc=N, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG, rowsum_a=db)
    close(dw, (dy.double().t() @ x.double()).cpu(), rtol=2e-6 * math.sqrt(K))
    close(db, dy.double().sum(0).cpu(), rtol=2e-6 * math.sqrt(K))


@pytest.mark.parametrize("layouts", ["fwd", "dgrad", "wgrad"])
def test_gemm_variants_bit_identical(mf, layouts):
    """Every pipelining variant (and hence the per-shape autotuner's pick) adds
    the k products in the same order: results must match bit for bit,
    including split-K and a K that is not a multiple of 32 -- the register-staged
    variants 0..7 and the direct-to-LDS variants 8..12 (gemm_glds_kernel.h; 12 is the
    128x192 tile of the N = 192 / 576 stage-0 shapes, here on N = 192 exactly and on ragged
    N) alike, with the bias-gradient row sums of an m-contiguous A (wgrad) too.  A K that
    is not a multiple of 4 cannot be staged by 16-B DMA: a forced direct-to-LDS variant
    falls back to the register kernel and still agrees."""
    from mdemi import _lib as L
    lib = L.load()
    for M, N, K in ((700, 300, 1000), (520, 264, 999), (384, 192, 320)):
        a = torch.randn(M, K, device=DEV)
        b = torch.randn(N, K, device=DEV)
        at, bt = a.t().contiguous(), b.t().contiguous()
        outs = []
        try:
            for v in range(13):
                L.check(lib.mdemi_gemm_set_variant(v, 8), "set_variant")
                for split in (1, 4, 5):
                    c = torch.empty(M, N, device=DEV)
                    rs = None
                    if layouts == "fwd":
                        mf.gemm(a, b, c, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
                                split_k=split)
                    elif layouts == "dgrad":
                        mf.gemm(a, bt, c, M, N, K, lda=K, ldb=N, ldc=N, a_layout=L.L_KCONTIG,
                                b_layout=L.L_MNCONTIG, split_k=split)
                    else:
                        rs = torch.empty(M, device=DEV)
                        mf.gemm(at, bt, c, M, N, K, lda=M, ldb=N, ldc=N, a_layout=L.L_MNCONTIG,
                                b_layout=L.L_MNCONTIG, split_k=split, rowsum_a=rs)
                    outs.append((v, split, c, rs))
        finally:
            lib.mdemi_gemm_set_variant(-1, 8)
        ref = (a.double() @ b.double().t()).float()
        for v, split, c, rs in outs:
            close(c, ref, rtol=1e-5 * math.sqrt(K))
            same = [o for o in outs if o[1] == split][0]
            assert torch.equal(c, same[2]), f"variant {v} split {split} differs bitwise (K={K})"
            if rs is not None:
                close(rs, a.double().sum(1).float(), rtol=1e-5 * math.sqrt(K))
                assert torch.equal(rs, same[3]), f"variant {v} split {split}: row sums differ bitwise (K={K})"


@pytest.mark.parametrize("layouts", ["fwd", "dgrad"])
def test_gemm_tail_split(mf, layouts):
    """Tail split (gemm_f32.hip tail_plan): 9600x3072x768 leaves a thin third round of
    128x128 tiles, so the rows holding them are cut at a 256-row boundary and split over K
    (combined by the last-arriving piece).  Every variant must agree bit for bit with the
    split on; rows above the cut equal the unsplit result bit for bit; all within the fp32
    bound of an fp64 product; the fused epilogue (bias, residual) runs after the combine."""
    from mdemi import _lib as L
    lib = L.load()
    M, N, K = 9600, 3072, 768
    g = torch.Generator(device=DEV).manual_seed(5)
    a = torch.randn(M, K, device=DEV, generator=g)
    b = torch.randn(N, K, device=DEV, generator=g)
    bt = b.t().contiguous()
    bias = torch.randn(N, device=DEV, generator=g)
    res = torch.randn(M, N, device=DEV, generator=g)

    def run(v, tail):
        L.check(lib.mdemi_gemm_set_variant(v, 8), "set_variant")
        L.check(lib.mdemi_gemm_set_options(tail, 1), "set_options")
        c = torch.empty(M, N, device=DEV)
        if layouts == "fwd":
            mf.gemm(a, b, c, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, split_k=1,
                    bias=bias, bias_mode=L.BIAS_COL, residual=res, ldres=N)
        else:
            mf.gemm(a, bt, c, M, N, K, lda=K, ldb=N, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG, split_k=1,
                    bias=bias, bias_mode=L.BIAS_COL, residual=res, ldres=N)
        return c

    try:
        plain = run(4, 0)
        outs = [(v, run(v, 1)) for v in (0, 1, 3, 4, 5, 6, 7)]
    finally:
        lib.mdemi_gemm_set_variant(-1, 8)
        lib.mdemi_gemm_set_options(1, 0)  # the defaults: tail split on, separate split-K reduce
    ref = (a.double() @ b.double().t() + bias.double() + res.double()).float()
    close(plain, ref, rtol=1e-5 * math.sqrt(K))
    m_split = _tail_plan_m_split(M, N, K, torch.cuda.get_device_properties(DEV).multi_processor_count)
    assert m_split > 0, "the shape must leave a thin last round on this device"
    for v, c in outs:
        close(c, ref, rtol=1e-5 * math.sqrt(K))
        assert torch.equal(c, outs[0][1]), f"variant {v} differs bitwise with the tail split"
    c = outs[0][1]
    assert torch.equal(c[:m_split], plain[:m_split]), "rows above the cut must be the unsplit result"
    assert not torch.equal(c[m_split:], plain[m_split:]), "tail rows were not split (plan did not engage)"


def _tail_plan_m_split(M, N, K, cus):
    """Host restatement of gemm_f32.hip tail_plan (batch 1, split_k 1): the first split row,
    0 when the plan does not engage.  The plan depends on the device's CU count, so which rows
    are split over K -- and hence their fp32 summation order -- differs between GPU SKUs."""
    cdiv = lambda a, b: -(-a // b)  # noqa: E731
    tm, tn = cdiv(M, 128), cdiv(N, 128)
    T, S = tm * tn, 3 * cus
    full, rem = T // S, T % S
    if full < 1 or rem == 0 or rem * 10 > S * 6:
        return 0
    m_split = (tm - cdiv(rem, tn)) // 2 * 256
    if m_split <= 0:
        return 0
    s = min(4, S // (cdiv(M - m_split, 128) * tn), cdiv(K, 32) // 2)
    return m_split if s >= 2 else 0


@pytest.mark.parametrize("layouts", ["fwd", "wgrad"])
def test_gemm_inline_combine_matches_reduce_kernel(mf, layouts):
    """Split-K slabs combined by the last-arriving piece of each tile (in split order) equal
    the separate gemm_splitk_reduce launch bit for bit, and repeated launches reuse the
    self-resetting tile counters.  wgrad: the bias-gradient row sums of the pieces are
    summed by the last arrivers too (no reduce launch), bit for bit as the reduce kernel
    sums them; with and without the fused bias epilogue (16-B epilogue and per-element
    path: N = 300 and N = 298)."""
    from mdemi import _lib as L
    lib = L.load()
    for M, N, K in ((700, 300, 5000), (700, 298, 5000)):
        a = torch.randn(M, K, device=DEV)
        b = torch.randn(N, K, device=DEV)
        bias = torch.randn(N, device=DEV)
        at, bt = a.t().contiguous(), b.t().contiguous()

        def run(inline):
            L.check(lib.mdemi_gemm_set_options(1, inline), "set_options")
            c = torch.empty(M, N, device=DEV)
            rs = None
            if layouts == "fwd":
                mf.gemm(a, b, c, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, split_k=6,
                        bias=bias, bias_mode=L.BIAS_COL)
            else:
                rs = torch.empty(M, device=DEV)
                mf.gemm(at, bt, c, M, N, K, lda=M, ldb=N, ldc=N, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
                        split_k=6, rowsum_a=rs)
            return c, rs

        try:
            k, krs = run(0)
            outs = [run(1) for _ in range(3)]
        finally:
            lib.mdemi_gemm_set_options(1, 0)  # the defaults: tail split on, separate split-K reduce
        want = a.double() @ b.double().t() + (bias.double() if layouts == "fwd" else 0.0)
        close(k, want.float(), rtol=1e-5 * math.sqrt(K))
        for c, rs in outs:
            assert torch.equal(c, k)
            if rs is not None:
                close(rs, a.double().sum(1).float(), rtol=1e-5 * math.sqrt(K))
                assert torch.equal(rs, krs)


def test_linear_and_mlp_drop_scale(mf):
    """DropPath fused into the proj / fc2 epilogue: y = res + s[sample] * (x W^T + b), and the
    branch gradients see s * dy while the residual's gradient is dy."""
    B, Lq, C, Hd = 3, 50, 64, 256
    x = rnd(B * Lq, C, seed=120)
    res = rnd(B * Lq, C, seed=121)
    w, bb = rnd(C, C, seed=122, scale=0.2), rnd(C, seed=123)
    w1, b1, w2, b2 = rnd(Hd, C, seed=124, scale=0.2), rnd(Hd, seed=125), rnd(C, Hd, seed=126, scale=0.1), rnd(C, seed=127)
    s = torch.tensor([2.0, 0.0, 2.0], dtype=torch.float64)
    srow = s.repeat_interleave(Lq).unsqueeze(1)
    dy = rnd(B * Lq, C, seed=128)
    # reference
    xr, rr = x.clone().requires_grad_(), res.clone().requires_grad_()
    wr, br_, w1r, b1r, w2r, b2r = (t.clone().requires_grad_() for t in (w, bb, w1, b1, w2, b2))
    y1 = rr + srow * (xr @ wr.t() + br_)
    y2 = y1 + srow * (F.gelu(y1 @ w1r.t() + b1r) @ w2r.t() + b2r)
    y2.backward(dy)
    # GPU
    g = lambda t: t.float().to(DEV).requires_grad_()
    xg, rg, wg, bg, w1g, b1g, w2g, b2g = (g(t) for t in (x, res, w, bb, w1, b1, w2, b2))
    sg = s.float().to(DEV)
    z1 = mf.linear(xg, wg, bg, residual=rg, drop_scale=sg)
    z2 = mf.mlp(z1, w1g, b1g, w2g, b2g, residual=z1, drop_scale=sg)
    z2.backward(dy.float().to(DEV))
    close(z2, y2, rtol=1e-5)
    for got, ref in ((xg, xr), (rg, rr), (wg, wr), (bg, br_), (w1g, w1r), (b1g, b1r), (w2g, w2r), (b2g, b2r)):
        close(got.grad, ref.grad, rtol=1e-4)


@pytest.mark.parametrize("cout,cin,kh,kw", [(8, 12, 3, 3), (5, 7, 5, 5), (16, 3, 4, 4), (6, 10, 1, 1), (4, 4, 1, 3)])
def test_conv_weight_layout(cout, cin, kh, kw):
    """mdemi_conv_weight_layout against the torch permutations it replaces (bit-exact)."""
    from mdemi import _lib as L
    from mdemi import functional as mf
    g = torch.Generator().manual_seed(cout * 100 + cin)
    w = torch.randn(cout, cin, kh, kw, generator=g)
    wg = w.to("cuda")
    assert torch.equal(mf.conv_weight_layout(wg, L.WL_OHWI).cpu(), w.permute(0, 2, 3, 1))
    assert torch.equal(mf.conv_weight_layout(wg, L.WL_DGRAD).cpu(), w.flip(2, 3).permute(2, 3, 0, 1))
    ohwi = w.permute(0, 2, 3, 1).contiguous()
    got = mf.conv_weight_layout(ohwi.to("cuda"), L.WL_OIHW, (cout, cin, kh, kw)).cpu()
    assert torch.equal(got, w)
