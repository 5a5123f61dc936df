"""Autograd wrappers over the libmdemi C ABI.

Every function here runs the hand-written gfx950 kernels through ``_lib``;
there is no eager/ATen fallback for the math (torch supplies device memory,
streams and the autograd tape).  Activations are channels-last: token-major
``[rows, C]`` tensors and NHWC feature maps.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib as L

# --------------------------------------------------------------------------
# helpers
# --------------------------------------------------------------------------


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("mdemi ops run on the GPU only; got a CPU tensor")
        if t is not None and t.dtype != torch.float32:
            raise ValueError(f"mdemi ops are fp32; got {t.dtype}")


def _c(t):
    return t if t is None or t.is_contiguous() else t.contiguous()


def _target_blocks():
    return 1024


def _split_for(M, N, K):
    """Split-K factor so that a long reduction still fills the chip."""
    tiles = math.ceil(M / 128) * math.ceil(N / 128)
    ktiles = math.ceil(K / 16)
    if tiles >= 512 or ktiles < 32:
        return 1
    split = min(max(1, _target_blocks() // tiles), ktiles // 16, 64)
    return max(1, split)


def gemm(A, B, C, M, N, K, *, lda, ldb, ldc, a_layout, b_layout, a_op=L.OP_NONE, b_op=L.OP_NONE,
         alpha=1.0, beta=0.0, bias=None, bias_mode=L.BIAS_NONE, act=L.ACT_NONE, aux=None, ldaux=0,
         residual=None, ldres=0, batch=1, a_bstride=0, b_bstride=0, c_bstride=0, aux_bstride=0,
         res_bstride=0, split_k=None, conv=None, preact=None, ldpre=0, pre_bstride=0, rowsum_a=None):
    d = L.GemmDesc()
    d.M, d.N, d.K, d.batch = M, N, K, batch
    d.A, d.lda, d.a_bstride, d.a_layout, d.a_op = A.data_ptr(), lda, a_bstride, a_layout, a_op
    d.B, d.ldb, d.b_bstride, d.b_layout, d.b_op = B.data_ptr(), ldb, b_bstride, b_layout, b_op
    d.C, d.ldc, d.c_bstride = C.data_ptr(), ldc, c_bstride
    d.alpha, d.beta = alpha, beta
    d.bias, d.bias_mode, d.act = (bias.data_ptr() if bias is not None else None), bias_mode, act
    d.aux, d.ldaux, d.aux_bstride = (aux.data_ptr() if aux is not None else None), ldaux, aux_bstride
    d.residual, d.ldres, d.res_bstride = (residual.data_ptr() if residual is not None else None), ldres, res_bstride
    d.split_k = split_k if split_k is not None else _split_for(M, N, K)
    if conv is not None:
        d.conv = conv
    if preact is not None:
        d.preact, d.ldpre, d.pre_bstride = preact.data_ptr(), ldpre, pre_bstride
    if rowsum_a is not None:
        d.rowsum_a = rowsum_a.data_ptr()
    lib = L.load()
    need = lib.mdemi_gemm_workspace_size(ctypes.byref(d))
    if need:
        ws = L.workspace(need, C.device, slot=1)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
    L.check(lib.mdemi_gemm_f32(ctypes.byref(d), L.stream()), "gemm_f32")
    return C


def colsum(x2d, out=None, accumulate=False):
    rows, cols = x2d.shape
    if out is None:
        out = torch.empty(cols, device=x2d.device, dtype=torch.float32)
    lib = L.load()
    ws = L.workspace(lib.mdemi_colsum_workspace_size(rows, cols), x2d.device)
    L.check(lib.mdemi_colsum_f32(x2d.data_ptr(), rows, cols, x2d.stride(0), out.data_ptr(), int(accumulate),
                                 ws.data_ptr(), L.stream()), "colsum")
    return out


# --------------------------------------------------------------------------
# Linear (nn.Linear) with GELU-on-load input and fused residual
# --------------------------------------------------------------------------


def linear_fwd_raw(x2, weight, bias, in_gelu=False, residual=None, act=L.ACT_NONE, out=None):
    M, K = x2.shape
    N = weight.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x2.device, dtype=torch.float32)
    gemm(x2, weight, out, M, N, K, lda=K, ldb=K, ldc=out.stride(0), a_layout=L.L_KCONTIG,
         b_layout=L.L_KCONTIG, a_op=L.OP_GELU if in_gelu else L.OP_NONE,
         bias=bias, bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE, act=act,
         residual=residual, ldres=(residual.stride(0) if residual is not None else 0), split_k=1)
    return out


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, in_gelu):
        _require_cuda(x, weight, bias, residual)
        K = x.shape[-1]
        x2 = _c(x).reshape(-1, K)
        res2 = _c(residual).reshape(x2.shape[0], -1) if residual is not None else None
        out = linear_fwd_raw(x2, _c(weight), bias, in_gelu=in_gelu, residual=res2)
        ctx.save_for_backward(x2, weight)
        ctx.in_gelu = in_gelu
        ctx.has_bias = bias is not None
        ctx.has_res = residual is not None
        ctx.xshape = x.shape
        return out.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        M, K = x2.shape
        N = weight.shape[0]
        dy2 = _c(dy).reshape(M, N)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, device=dy.device, dtype=torch.float32)
            # dX[M,K] = dY[M,N] . W[N,K]  (times gelu'(h) when the forward read gelu(h))
            gemm(dy2, weight, dx, M, K, N, lda=N, ldb=K, ldc=K, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG,
                 act=L.ACT_GELU_GRAD if ctx.in_gelu else L.ACT_NONE, aux=x2 if ctx.in_gelu else None,
                 ldaux=K)
            dx = dx.view(ctx.xshape)
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        if want_db:
            db = torch.empty(N, device=dy.device, dtype=torch.float32)
        if ctx.needs_input_grad[1]:
            dw = torch.empty(N, K, device=dy.device, dtype=torch.float32)
            # dW[N,K] = dY^T . X  (reduction over the M rows; split-K slabs); db = dY^T 1 rides along
            gemm(dy2, x2, dw, N, K, M, lda=N, ldb=K, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
                 b_op=L.OP_GELU if ctx.in_gelu else L.OP_NONE, rowsum_a=db)
        elif want_db:
            colsum(dy2, out=db)
        dres = dy if ctx.has_res and ctx.needs_input_grad[3] else None
        return dx, dw, db, dres, None


def linear(x, weight, bias=None, residual=None, in_gelu=False):
    """y = (gelu(x) if in_gelu else x) @ W^T + b (+ residual)."""
    return _LinearFn.apply(x, weight, bias, residual, in_gelu)


class _MlpFn(torch.autograd.Function):
    """fc1 -> GELU -> fc2 (+ residual), Swin/NeW-CRF Mlp (swin_transformer.py:11-29).

    fc1's epilogue writes both h (pre-activation) and g = gelu(h): HBM is
    plentiful and one extra [rows, 4C] store is far cheaper than recomputing
    gelu in fc2's operand loader for every N-tile.  Backward: fc2's dgrad
    epilogue multiplies by gelu'(h) (reading h), so dh never exists unfused."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, residual):
        _require_cuda(x, w1, b1, w2, b2, residual)
        K = x.shape[-1]
        x2 = _c(x).reshape(-1, K)
        M = x2.shape[0]
        Hd, N = w1.shape[0], w2.shape[0]
        h = torch.empty(M, Hd, device=x.device, dtype=torch.float32)
        g = torch.empty(M, Hd, device=x.device, dtype=torch.float32)
        gemm(x2, _c(w1), g, M, Hd, K, lda=K, ldb=K, ldc=Hd, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
             bias=b1, bias_mode=L.BIAS_COL if b1 is not None else L.BIAS_NONE, act=L.ACT_GELU,
             preact=h, ldpre=Hd, split_k=1)
        res2 = _c(residual).reshape(M, N) if residual is not None else None
        out = linear_fwd_raw(g, _c(w2), b2, residual=res2)
        ctx.save_for_backward(x2, w1, w2, h, g)
        ctx.flags = (b1 is not None, b2 is not None, residual is not None)
        ctx.xshape = x.shape
        return out.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w1, w2, h, g = ctx.saved_tensors
        has_b1, has_b2, has_res = ctx.flags
        M, K = x2.shape
        Hd, N = w1.shape[0], w2.shape[0]
        dy2 = _c(dy).reshape(M, N)
        dev = dy.device
        dw2 = torch.empty(N, Hd, device=dev, dtype=torch.float32)
        db2 = torch.empty(N, device=dev, dtype=torch.float32) if has_b2 else None
        gemm(dy2, g, dw2, N, Hd, M, lda=N, ldb=Hd, ldc=Hd, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
             rowsum_a=db2)
        dh = torch.empty(M, Hd, device=dev, dtype=torch.float32)
        gemm(dy2, w2, dh, M, Hd, N, lda=N, ldb=Hd, ldc=Hd, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG,
             act=L.ACT_GELU_GRAD, aux=h, ldaux=Hd)
        del h, g
        dw1 = torch.empty(Hd, K, device=dev, dtype=torch.float32)
        db1 = torch.empty(Hd, device=dev, dtype=torch.float32) if has_b1 else None
        gemm(dh, x2, dw1, Hd, K, M, lda=Hd, ldb=K, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
             rowsum_a=db1)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, device=dev, dtype=torch.float32)
            gemm(dh, w1, dx, M, K, Hd, lda=Hd, ldb=K, ldc=K, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG)
            dx = dx.view(ctx.xshape)
        dres = dy if has_res and ctx.needs_input_grad[5] else None
        return dx, dw1, db1, dw2, db2, dres


def mlp(x, w1, b1, w2, b2, residual=None):
    """fc2(gelu(fc1(x))) (+ residual) with nn.GELU (exact erf)."""
    return _MlpFn.apply(x, w1, b1, w2, b2, residual)


# --------------------------------------------------------------------------
# Conv2d on NHWC activations (implicit im2col on the GEMM operand loader)
# --------------------------------------------------------------------------


def _geom(n, h, w, c, oh, ow, kh, kw, stride, pad, pad_mode):
    g = L.ConvGeom()
    g.n, g.h, g.w, g.c, g.oh, g.ow = n, h, w, c, oh, ow
    g.kh, g.kw, g.stride, g.pad, g.pad_mode = kh, kw, stride, pad, pad_mode
    return g


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, pad_mode, act):
        _require_cuda(x, weight, bias)
        x = _c(x)
        n, h, w, c = x.shape
        cout, cin, kh, kw = weight.shape
        if cin != c:
            raise ValueError(f"conv2d: input has {c} channels, weight expects {cin}")
        oh = (h + 2 * pad - kh) // stride + 1
        ow = (w + 2 * pad - kw) // stride + 1
        M, K = n * oh * ow, kh * kw * c
        out = torch.empty(n, oh, ow, cout, device=x.device, dtype=torch.float32)
        wf = weight.permute(0, 2, 3, 1).reshape(cout, K).contiguous()
        pointwise = kh == 1 and kw == 1 and stride == 1 and pad == 0
        if pointwise:
            gemm(x, wf, out, M, cout, K, lda=c, ldb=K, ldc=cout, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
                 bias=bias, bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE, act=act, split_k=1)
        else:
            if c % 4:
                raise ValueError("conv2d: implicit-GEMM path needs C % 4 == 0")
            gemm(x, wf, out, M, cout, K, lda=0, ldb=K, ldc=cout, a_layout=L.L_CONV, b_layout=L.L_KCONTIG,
                 bias=bias, bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE, act=act,
                 conv=_geom(n, h, w, c, oh, ow, kh, kw, stride, pad, pad_mode))
        ctx.save_for_backward(x, weight, out if act != L.ACT_NONE else None)
        ctx.cfg = (stride, pad, pad_mode, act, bias is not None, pointwise)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        stride, pad, pad_mode, act, has_bias, pointwise = ctx.cfg
        dy = _c(dy)
        if act != L.ACT_NONE:
            if act != L.ACT_RELU:
                raise NotImplementedError("conv2d backward: only ReLU epilogue supported")
            g = torch.empty_like(dy)
            L.call("mdemi_elementwise", L.EW_ACT_BWD, y.data_ptr(), dy.data_ptr(), g.data_ptr(), dy.numel(),
                   float(L.ACT_RELU), 0.0, L.stream())
            dy = g
        n, h, w, c = x.shape
        cout, cin, kh, kw = weight.shape
        _, oh, ow, _ = dy.shape
        M, K = n * oh * ow, kh * kw * c
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if pointwise:
                dx = torch.empty_like(x)
                gemm(dy, weight.reshape(cout, cin), dx, M, c, cout, lda=cout, ldb=cin, ldc=c,
                     a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG)
            else:
                if stride != 1 or pad_mode != L.PAD_ZERO:
                    raise NotImplementedError("conv2d dgrad: stride 1, zero padding only")
                # dX = conv(dY, flip(W)^T) with pad k-1-p:  Wd[(ky,kx,co)][c] = W[co][c][k-1-ky][k-1-kx]
                wd = weight.flip(2, 3).permute(2, 3, 0, 1).reshape(kh * kw * cout, cin).contiguous()
                dx = torch.empty_like(x)
                gemm(dy, wd, dx, n * h * w, c, kh * kw * cout, lda=0, ldb=cin, ldc=c, a_layout=L.L_CONV,
                     b_layout=L.L_MNCONTIG, split_k=1,
                     conv=_geom(n, oh, ow, cout, h, w, kh, kw, 1, kh - 1 - pad, L.PAD_ZERO))
        want_db = has_bias and ctx.needs_input_grad[2]
        if want_db:
            db = torch.empty(cout, device=dy.device, dtype=torch.float32)
        if ctx.needs_input_grad[1]:
            dwf = torch.empty(cout, K, device=dy.device, dtype=torch.float32)
            if pointwise:
                gemm(dy, x, dwf, cout, K, M, lda=cout, ldb=c, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
                     rowsum_a=db)
            else:
                gemm(dy, x, dwf, cout, K, M, lda=cout, ldb=0, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_CONV,
                     conv=_geom(n, h, w, c, oh, ow, kh, kw, stride, pad, pad_mode), rowsum_a=db)
            dw = dwf.view(cout, kh, kw, cin).permute(0, 3, 1, 2).contiguous()
        elif want_db:
            colsum(dy.reshape(-1, cout), out=db)
        return dx, dw, db, None, None, None, None


class _HeadConvFn(torch.autograd.Function):
    """KxK 'same' conv with a single output channel (DispHead.conv1)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        _require_cuda(x, weight, bias)
        x, weight = _c(x), _c(weight)
        n, h, w, c = x.shape
        k = weight.shape[-1]
        y = torch.empty(n, h, w, 1, device=x.device, dtype=torch.float32)
        L.call("mdemi_headconv_fwd", x.data_ptr(), weight.data_ptr(), L.ptr(bias), y.data_ptr(), n, h, w, c, k,
               k // 2, L.stream())
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = _c(dy)
        n, h, w, c = x.shape
        k = weight.shape[-1]
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(weight) if ctx.needs_input_grad[1] else None
        db = torch.empty(1, device=x.device, dtype=torch.float32) if ctx.has_bias and ctx.needs_input_grad[2] else None
        lib = L.load()
        ws = L.workspace(lib.mdemi_headconv_wgrad_workspace_size(n, h, w, c, k), x.device)
        L.check(lib.mdemi_headconv_bwd(dy.data_ptr(), x.data_ptr(), weight.data_ptr(), L.ptr(dx), L.ptr(dw), L.ptr(db),
                                       n, h, w, c, k, k // 2, ws.data_ptr(), L.stream()), "headconv_bwd")
        return dx, dw, db


def conv2d_nhwc(x, weight, bias=None, stride=1, pad=0, pad_mode=L.PAD_ZERO, act=L.ACT_NONE):
    if weight.shape[0] == 1 and stride == 1 and pad_mode == L.PAD_ZERO and act == L.ACT_NONE and \
            2 * pad == weight.shape[-1] - 1 and weight.shape[-1] <= 3 and x.shape[-1] % 4 == 0 and \
            x.shape[-1] <= 128:
        return _HeadConvFn.apply(x, weight, bias)
    return _Conv2dFn.apply(x, weight, bias, stride, pad, pad_mode, act)


class _PatchEmbedFn(torch.autograd.Function):
    """Conv with kernel == stride (PatchEmbed, swin_transformer.py:414,429) on an NCHW image:
    patchify sweep + GEMM.  Output NHWC.  The image gets no gradient."""

    @staticmethod
    def forward(ctx, img, weight, bias):
        _require_cuda(img, weight, bias)
        img = _c(img)
        n, c, h, w = img.shape
        cout, cin, p, _ = weight.shape
        hp, wp = -(-h // p), -(-w // p)
        K = c * p * p
        cols = torch.empty(n * hp * wp, K, device=img.device, dtype=torch.float32)
        L.call("mdemi_patchify_nchw", img.data_ptr(), cols.data_ptr(), n, c, h, w, p, 0, L.stream())
        out = torch.empty(n, hp, wp, cout, device=img.device, dtype=torch.float32)
        gemm(cols, _c(weight).reshape(cout, K), out, n * hp * wp, cout, K, lda=K, ldb=K, ldc=cout,
             a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, bias=bias,
             bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE, split_k=1)
        ctx.save_for_backward(cols, weight)
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, dy):
        cols, weight = ctx.saved_tensors
        cout = weight.shape[0]
        M, K = cols.shape
        dy2 = _c(dy).reshape(M, cout)
        dw = torch.empty(cout, K, device=dy.device, dtype=torch.float32)
        db = torch.empty(cout, device=dy.device, dtype=torch.float32) if ctx.has_bias else None
        gemm(dy2, cols, dw, cout, K, M, lda=cout, ldb=K, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
             rowsum_a=db)
        return None, dw.view_as(weight), db


def patch_embed(img_nchw, weight, bias):
    return _PatchEmbedFn.apply(img_nchw, weight, bias)


# --------------------------------------------------------------------------
# LayerNorm
# --------------------------------------------------------------------------


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        _require_cuda(x, weight, bias)
        x = _c(x)
        C = x.shape[-1]
        rows = x.numel() // C
        y = torch.empty_like(x)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        L.call("mdemi_layernorm_fwd", x.data_ptr(), weight.data_ptr(), bias.data_ptr(), y.data_ptr(),
               mean.data_ptr(), rstd.data_ptr(), rows, C, float(eps), L.stream())
        ctx.save_for_backward(x, weight, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, mean, rstd = ctx.saved_tensors
        dy = _c(dy)
        C = x.shape[-1]
        rows = x.numel() // C
        dx = torch.empty_like(x)
        dg = torch.empty(C, device=x.device, dtype=torch.float32)
        db = torch.empty(C, device=x.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_layernorm_bwd_workspace_size(rows, C), x.device)
        L.check(lib.mdemi_layernorm_bwd(dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                        weight.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), rows, C, 0,
                                        ws.data_ptr(), L.stream()), "layernorm_bwd")
        return dx, dg, db, None


def layer_norm(x, weight, bias, eps=1e-5):
    return _LayerNormFn.apply(x, weight, bias, eps)


# --------------------------------------------------------------------------
# (Shifted-)window attention
# --------------------------------------------------------------------------


class _WindowAttnFn(torch.autograd.Function):
    """q/k come from `qk` ([rows, >=2C]: q at col 0, k at col C); v from `v` ([rows, ...] at
    column v_off).  Pad tokens read qk_bias / v_bias (None -> zeros)."""

    @staticmethod
    def forward(ctx, qk, qk_bias, v, v_bias, rpb, geom):
        _require_cuda(qk, qk_bias, v, v_bias, rpb)
        B, H, W, heads, window, shift, scale, C, v_off = geom
        rows = B * H * W
        out = torch.empty(rows, C, device=qk.device, dtype=torch.float32)
        d = L.WinAttnDesc()
        d.B, d.H, d.W, d.heads, d.head_dim, d.window, d.shift = B, H, W, heads, C // heads, window, shift
        d.scale = scale
        d.q, d.k, d.qk_ld = qk.data_ptr(), qk.data_ptr() + 4 * C, qk.stride(0)
        d.q_pad = qk_bias.data_ptr() if qk_bias is not None else None
        d.k_pad = qk_bias.data_ptr() + 4 * C if qk_bias is not None else None
        d.v, d.v_ld = v.data_ptr() + 4 * v_off, v.stride(0)
        d.v_pad = v_bias.data_ptr() + 4 * v_off if v_bias is not None else None
        d.rpb_table = rpb.data_ptr()
        d.out, d.out_ld = out.data_ptr(), C
        ws = window
        nwin = B * (-(-H // ws)) * (-(-W // ws))
        lse = torch.empty(nwin, heads, ws * ws, device=qk.device, dtype=torch.float32)
        d.lse = lse.data_ptr()
        lib = L.load()
        ws_f = L.workspace(lib.mdemi_winattn_fwd_workspace_size(ctypes.byref(d)), qk.device)
        d.workspace, d.workspace_bytes = ws_f.data_ptr(), ws_f.numel()
        L.check(lib.mdemi_winattn_fwd(ctypes.byref(d), L.stream()), "winattn_fwd")
        ctx.save_for_backward(qk, qk_bias, v, v_bias, rpb, out, lse)
        ctx.geom = geom
        ctx.has_qkb = qk_bias is not None
        ctx.has_vb = v_bias is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        qk, qk_bias, v, v_bias, rpb, out, lse = ctx.saved_tensors
        B, H, W, heads, window, shift, scale, C, v_off = ctx.geom
        dout = _c(dout)
        dqk = torch.empty_like(qk)
        same = v.data_ptr() == qk.data_ptr()
        if same:
            dv_t = dqk
        else:
            dv_t = torch.empty_like(v)
        if dqk.shape[1] > 2 * C and not same:
            dqk[:, 2 * C:].zero_()
        if dv_t.shape[1] > C and not same:
            dv_t.zero_()
        d_rpb = torch.empty_like(rpb)
        pad_g = torch.zeros(3, C, device=qk.device, dtype=torch.float32)
        d = L.WinAttnDesc()
        d.B, d.H, d.W, d.heads, d.head_dim, d.window, d.shift = B, H, W, heads, C // heads, window, shift
        d.scale = scale
        d.q, d.k, d.qk_ld = qk.data_ptr(), qk.data_ptr() + 4 * C, qk.stride(0)
        d.q_pad = qk_bias.data_ptr() if qk_bias is not None else None
        d.k_pad = qk_bias.data_ptr() + 4 * C if qk_bias is not None else None
        d.v, d.v_ld = v.data_ptr() + 4 * v_off, v.stride(0)
        d.v_pad = v_bias.data_ptr() + 4 * v_off if v_bias is not None else None
        d.rpb_table = rpb.data_ptr()
        d.out, d.out_ld, d.lse = out.data_ptr(), C, lse.data_ptr()
        d.dout = dout.data_ptr()
        d.dq, d.dk, d.dqk_ld = dqk.data_ptr(), dqk.data_ptr() + 4 * C, dqk.stride(0)
        d.dv, d.dv_ld = dv_t.data_ptr() + 4 * v_off, dv_t.stride(0)
        d.d_rpb_table = d_rpb.data_ptr()
        d.dq_pad, d.dk_pad, d.dv_pad = pad_g[0].data_ptr(), pad_g[1].data_ptr(), pad_g[2].data_ptr()
        lib = L.load()
        need = lib.mdemi_winattn_bwd_workspace_size(ctypes.byref(d))
        ws = L.workspace(need, qk.device)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
        L.check(lib.mdemi_winattn_bwd(ctypes.byref(d), L.stream()), "winattn_bwd")
        dqk_bias = dv_bias = None
        if ctx.has_qkb:
            dqk_bias = torch.zeros_like(qk_bias)
            dqk_bias[:C] = pad_g[0]
            dqk_bias[C:2 * C] = pad_g[1]
            if same and ctx.has_vb:
                dqk_bias[v_off:v_off + C] += pad_g[2]
        if ctx.has_vb and not same:
            dv_bias = torch.zeros_like(v_bias)
            dv_bias[v_off:v_off + C] = pad_g[2]
        if same:
            return dqk, dqk_bias, None, None, d_rpb, None
        return dqk, dqk_bias, dv_t, dv_bias, d_rpb, None


def window_attention(qk, qk_bias, v, v_bias, rpb_table, B, H, W, heads, window, shift, scale, C, v_off=0):
    """Swin: qk = v = qkv output [rows,3C], qk_bias = v_bias = qkv.bias, v_off = 2C.
    NeW-CRF: qk = qk output [rows,2C] with its bias; v [rows,C] padded with zeros (v_bias None)."""
    geom = (B, H, W, heads, window, shift, float(scale), C, v_off)
    if v is qk:
        # one tensor feeds q, k and v: pass it once so autograd sums its gradient
        return _WindowAttnFn.apply(qk, qk_bias, qk, qk_bias if v_bias is not None else None, rpb_table, geom)
    return _WindowAttnFn.apply(qk, qk_bias, v, v_bias, rpb_table, geom)


# --------------------------------------------------------------------------
# Adaptive-bin depth head
# --------------------------------------------------------------------------


class _BinHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, centers, do_softmax):
        _require_cuda(logits, centers)
        logits = _c(logits)
        centers = _c(centers)
        B, K = logits.shape[:2]
        HW = logits[0, 0].numel()
        pred = torch.empty(B, 1, *logits.shape[2:], device=logits.device, dtype=torch.float32)
        stats = torch.empty(B, 2, HW, device=logits.device, dtype=torch.float32) if do_softmax else None
        L.call("mdemi_binhead_fwd", logits.data_ptr(), centers.data_ptr(), pred.data_ptr(), L.ptr(stats), None,
               B, K, HW, int(do_softmax), L.stream())
        ctx.save_for_backward(logits, centers, pred, stats)
        ctx.do_softmax = do_softmax
        return pred

    @staticmethod
    def backward(ctx, dpred):
        logits, centers, pred, stats = ctx.saved_tensors
        dpred = _c(dpred)
        B, K = logits.shape[:2]
        HW = logits[0, 0].numel()
        dlogits = torch.empty_like(logits)
        dcenters = torch.empty(B, K, device=logits.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_binhead_bwd_workspace_size(B, K, HW), logits.device)
        L.check(lib.mdemi_binhead_bwd(logits.data_ptr(), centers.data_ptr(), pred.data_ptr(), L.ptr(stats),
                                      dpred.data_ptr(), dlogits.data_ptr(), dcenters.data_ptr(), B, K, HW,
                                      int(ctx.do_softmax), ws.data_ptr(), L.stream()), "binhead_bwd")
        return dlogits, dcenters.view_as(centers), None


def bin_head(logits, centers, do_softmax=True):
    """pred[b,0,...] = sum_k softmax_k(logits)[b,k,...] * centers[b,k]   (NCHW logits)."""
    return _BinHeadFn.apply(logits, centers.reshape(logits.shape[0], logits.shape[1]), do_softmax)


# --------------------------------------------------------------------------
# SILog loss
# --------------------------------------------------------------------------


class _SILogFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, min_depth, alpha, beta, per_image, unbiased):
        _require_cuda(pred, gt)
        pred = _c(pred)
        gt = _c(gt)
        B = pred.shape[0]
        HW = pred[0].numel()
        G = B if per_image else 1
        loss = torch.empty(1, device=pred.device, dtype=torch.float32)
        stats = torch.empty(G, 4, device=pred.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_silog_workspace_size(B, HW), pred.device, slot=2)
        L.check(lib.mdemi_silog_fwd(pred.data_ptr(), gt.data_ptr(), loss.data_ptr(), stats.data_ptr(), B, HW,
                                    float(min_depth), float(alpha), float(beta), int(per_image), int(unbiased),
                                    ws.data_ptr(), L.stream()), "silog_fwd")
        ctx.save_for_backward(pred, gt, stats)
        ctx.cfg = (min_depth, alpha, beta, per_image, unbiased)
        return loss[0]

    @staticmethod
    def backward(ctx, dloss):
        pred, gt, stats = ctx.saved_tensors
        min_depth, alpha, beta, per_image, unbiased = ctx.cfg
        B = pred.shape[0]
        HW = pred[0].numel()
        dpred = torch.empty_like(pred)
        dl = _c(dloss.reshape(1).to(torch.float32))
        L.call("mdemi_silog_bwd", pred.data_ptr(), gt.data_ptr(), stats.data_ptr(), dl.data_ptr(),
               dpred.data_ptr(), B, HW, float(min_depth), float(alpha), float(beta), int(per_image),
               int(unbiased), L.stream())
        return dpred, None, None, None, None, None, None


def silog_loss(pred, gt, min_depth=1e-3, alpha=10.0, beta=0.15, per_image=False, unbiased=False):
    return _SILogFn.apply(pred, gt, min_depth, alpha, beta, per_image, unbiased)


# --------------------------------------------------------------------------
# Resampling / layout
# --------------------------------------------------------------------------


class _BilinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow, align_corners, sh, sw):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n, oh, ow, c, device=x.device, dtype=torch.float32)
        L.call("mdemi_bilinear_fwd", x.data_ptr(), y.data_ptr(), n, h, w, c, oh, ow, int(align_corners),
               float(sh), float(sw), c, c, L.stream())
        ctx.cfg = (n, h, w, c, oh, ow, align_corners, sh, sw)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, oh, ow, align_corners, sh, sw = ctx.cfg
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_bilinear_bwd", dy.data_ptr(), dx.data_ptr(), n, h, w, c, oh, ow, int(align_corners),
               float(sh), float(sw), c, c, 0, L.stream())
        return dx, None, None, None, None, None


def interpolate_bilinear(x_nhwc, size=None, scale_factor=None, align_corners=False):
    n, h, w, c = x_nhwc.shape
    if size is not None:
        oh, ow = size
        sh = sw = 0.0
    else:
        sh = sw = float(scale_factor)
        oh, ow = int(math.floor(h * sh)), int(math.floor(w * sw))
        if align_corners:
            sh = sw = 0.0
    return _BilinearFn.apply(x_nhwc, oh, ow, align_corners, sh, sw)


class _PixelShuffleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n, h * r, w * r, c // (r * r), device=x.device, dtype=torch.float32)
        L.call("mdemi_pixel_shuffle_nhwc", x.data_ptr(), y.data_ptr(), n, h, w, c, r, 0, L.stream())
        ctx.cfg = (n, h, w, c, r)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, r = ctx.cfg
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_pixel_shuffle_nhwc", dy.data_ptr(), dx.data_ptr(), n, h, w, c, r, 1, L.stream())
        return dx, None


def pixel_shuffle_nhwc(x, r):
    return _PixelShuffleFn.apply(x, r)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n, oh, ow, c, device=x.device, dtype=torch.float32)
        L.call("mdemi_adaptive_avgpool_fwd", x.data_ptr(), y.data_ptr(), n, h, w, c, oh, ow, L.stream())
        ctx.cfg = (n, h, w, c, oh, ow)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, oh, ow = ctx.cfg
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_adaptive_avgpool_bwd", dy.data_ptr(), dx.data_ptr(), n, h, w, c, oh, ow, L.stream())
        return dx, None, None


def adaptive_avg_pool_nhwc(x, out_size):
    oh, ow = (out_size, out_size) if isinstance(out_size, int) else out_size
    return _AvgPoolFn.apply(x, oh, ow)


class _LayoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, to_nhwc):
        _require_cuda(x)
        x = _c(x)
        ctx.to_nhwc = to_nhwc
        if to_nhwc:
            n, c, h, w = x.shape
            y = torch.empty(n, h, w, c, device=x.device, dtype=torch.float32)
            L.call("mdemi_nchw_to_nhwc", x.data_ptr(), y.data_ptr(), n, c, h * w, L.stream())
        else:
            n, h, w, c = x.shape
            y = torch.empty(n, c, h, w, device=x.device, dtype=torch.float32)
            L.call("mdemi_nhwc_to_nchw", x.data_ptr(), y.data_ptr(), n, c, h * w, L.stream())
        return y

    @staticmethod
    def backward(ctx, dy):
        return _LayoutFn.apply(dy, not ctx.to_nhwc), None


def nchw_to_nhwc(x):
    return _LayoutFn.apply(x, True)


def nhwc_to_nchw(x):
    return _LayoutFn.apply(x, False)


# --------------------------------------------------------------------------
# BatchNorm / GroupNorm (training-mode statistics) with fused activation
# --------------------------------------------------------------------------


class _ChNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, groups, is_bn, eps, act):
        _require_cuda(x, weight, bias)
        x = _c(x)
        n = x.shape[0]
        c = x.shape[-1]
        hw = x[0].numel() // c
        y = torch.empty_like(x)
        nstat = c if is_bn else n * groups
        mean = torch.empty(nstat, device=x.device, dtype=torch.float32)
        rstd = torch.empty(nstat, device=x.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_chnorm_workspace_size(n, hw, c, groups, int(is_bn)), x.device)
        L.check(lib.mdemi_chnorm_fwd(x.data_ptr(), weight.data_ptr(), bias.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                     rstd.data_ptr(), n, hw, c, groups, int(is_bn), float(eps), act, ws.data_ptr(),
                                     L.stream()), "chnorm_fwd")
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.cfg = (groups, is_bn, act)
        ctx.mark_non_differentiable(mean, rstd)
        return y, mean, rstd

    @staticmethod
    def backward(ctx, dy, _dm, _dr):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        groups, is_bn, act = ctx.cfg
        dy = _c(dy)
        n = x.shape[0]
        c = x.shape[-1]
        hw = x[0].numel() // c
        dx = torch.empty_like(x)
        dg = torch.empty(c, device=x.device, dtype=torch.float32)
        db = torch.empty(c, device=x.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_chnorm_workspace_size(n, hw, c, groups, int(is_bn)), x.device)
        L.check(lib.mdemi_chnorm_bwd(dy.data_ptr(), x.data_ptr(), None, mean.data_ptr(), rstd.data_ptr(),
                                     weight.data_ptr(), bias.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(),
                                     n, hw, c, groups, int(is_bn), act, ws.data_ptr(), L.stream()), "chnorm_bwd")
        return dx, dg, db, None, None, None, None


def batch_norm_nhwc(x, weight, bias, eps=1e-5, act=L.ACT_NONE):
    """Training-mode BatchNorm2d over an NHWC map; returns (y, batch_mean, batch_rstd)."""
    return _ChNormFn.apply(x, weight, bias, x.shape[-1], True, eps, act)


def group_norm_nhwc(x, weight, bias, groups, eps=1e-5, act=L.ACT_NONE):
    y, _, _ = _ChNormFn.apply(x, weight, bias, groups, False, eps, act)
    return y


# --------------------------------------------------------------------------
# elementwise
# --------------------------------------------------------------------------


class _SigmoidScaleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        _require_cuda(x)
        x = _c(x)
        y = torch.empty_like(x)
        L.call("mdemi_elementwise", L.EW_SIGMOID_SCALE, x.data_ptr(), None, y.data_ptr(), x.numel(), float(s), 0.0,
               L.stream())
        ctx.save_for_backward(x)
        ctx.s = s
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = _c(dy)
        dx = torch.empty_like(x)
        L.call("mdemi_elementwise", L.EW_SIGMOID_SCALE_BWD, x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(),
               float(ctx.s), 0.0, L.stream())
        return dx, None


def sigmoid_scale(x, s=1.0):
    return _SigmoidScaleFn.apply(x, s)


class _AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        _require_cuda(a, b)
        a, b = _c(a), _c(b)
        y = torch.empty_like(a)
        L.call("mdemi_elementwise", L.EW_ADD, a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), 0.0, 0.0,
               L.stream())
        return y

    @staticmethod
    def backward(ctx, dy):
        return dy, dy


def add(a, b):
    return _AddFn.apply(a, b)


# --------------------------------------------------------------------------
# PatchMerging gather, channel concat, stochastic depth
# --------------------------------------------------------------------------


class _SpaceToDepth2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n, (h + 1) // 2, (w + 1) // 2, 4 * c, device=x.device, dtype=torch.float32)
        L.call("mdemi_space_to_depth2", x.data_ptr(), y.data_ptr(), n, h, w, c, 0, L.stream())
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c = ctx.shape
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_space_to_depth2", dx.data_ptr(), dy.data_ptr(), n, h, w, c, 1, L.stream())
        return dx


def space_to_depth2(x_nhwc):
    """PatchMerging's x0..x3 gather + cat (swin_transformer.py:272-284), NHWC."""
    return _SpaceToDepth2Fn.apply(x_nhwc)


def _copy2d(src2, dst2, accumulate=False):
    rows, cols = src2.shape
    L.call("mdemi_copy2d", src2.data_ptr(), src2.stride(0), dst2.data_ptr(), dst2.stride(0), rows, cols,
           int(accumulate), L.stream())


class _ConcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        _require_cuda(*xs)
        xs = [_c(x) for x in xs]
        lead = xs[0].shape[:-1]
        widths = [x.shape[-1] for x in xs]
        out = torch.empty(*lead, sum(widths), device=xs[0].device, dtype=torch.float32)
        o2 = out.view(-1, out.shape[-1])
        off = 0
        for x, wd in zip(xs, widths):
            _copy2d(x.view(-1, wd), o2[:, off:off + wd])
            off += wd
        ctx.widths = widths
        return out

    @staticmethod
    def backward(ctx, dy):
        dy = _c(dy)
        d2 = dy.view(-1, dy.shape[-1])
        grads = []
        off = 0
        for wd in ctx.widths:
            g = torch.empty(*dy.shape[:-1], wd, device=dy.device, dtype=torch.float32)
            _copy2d(d2[:, off:off + wd], g.view(-1, wd))
            grads.append(g)
            off += wd
        return tuple(grads)


def concat_channels(xs):
    """torch.cat(dim=1) of NCHW maps == channel concat of NHWC maps."""
    return _ConcatFn.apply(*xs)


class _DropPathAddFn(torch.autograd.Function):
    """y = res + branch * scale[sample]  (timm DropPath with scale = keep / (1 - p))."""

    @staticmethod
    def forward(ctx, res, branch, scale):
        res, branch = _c(res), _c(branch)
        y = torch.empty_like(branch)
        per = branch.numel() // scale.numel()
        L.call("mdemi_rowscale_add", res.data_ptr(), branch.data_ptr(), scale.data_ptr(), y.data_ptr(), per,
               branch.numel(), L.stream())
        ctx.save_for_backward(scale)
        ctx.per = per
        return y

    @staticmethod
    def backward(ctx, dy):
        (scale,) = ctx.saved_tensors
        dy = _c(dy)
        db = torch.empty_like(dy)
        L.call("mdemi_rowscale_add", None, dy.data_ptr(), scale.data_ptr(), db.data_ptr(), ctx.per, dy.numel(),
               L.stream())
        return dy, db, None


def drop_path_add(res, branch, drop_prob, training):
    if drop_prob == 0.0 or not training:
        return add(res, branch)
    keep = 1.0 - drop_prob
    scale = torch.empty(branch.shape[0], device=branch.device, dtype=torch.float32).bernoulli_(keep).div_(keep)
    return _DropPathAddFn.apply(res, branch, scale)


def batch_norm_eval_nhwc(x, weight, bias, running_mean, running_var, eps=1e-5, act=L.ACT_NONE):
    """Inference BatchNorm2d (running statistics); no autograd."""
    _require_cuda(x)
    x = _c(x)
    n, c = x.shape[0], x.shape[-1]
    hw = x[0].numel() // c
    rstd = torch.rsqrt(running_var + eps)
    y = torch.empty_like(x)
    L.call("mdemi_chnorm_apply", x.data_ptr(), weight.data_ptr(), bias.data_ptr(), running_mean.data_ptr(),
           rstd.data_ptr(), y.data_ptr(), n, hw, c, c, 1, act, L.stream())
    return y
