"""bf16 mixed-precision emulation for the oracles (TEST INFRASTRUCTURE ONLY -- see
oracle/__init__.py).

Inside ``enabled()`` the GEMM-shaped ops of the oracles -- conv2d with groups == 1,
linear, matmul -- round both operands to bf16 (round-to-nearest-even) before the product,
in the forward and in each backward product, exactly as mdemi's precision="bf16" GEMMs
do (mdemi_gemm_bf16: every operand of every GEMM rounded, fp32 accumulation): the
forward rounds (x, w); the input gradient rounds (dy, w); the weight gradient rounds
(dy, x); a bias gradient sums the UNROUNDED dy (the GEMM's fp32 row sums).  Everything
else (norms, softmax, activations, depthwise convs, squeeze-excite) stays at the oracle's
precision, as it does on the GPU.  The products themselves run in the oracle's dtype
(fp64 or fp32), so the fp64 run is the exact value of the bf16-operand computation.
Outside the context the three functions are torch's own."""
import contextlib

import torch
import torch.nn.functional as F
from torch.nn import grad as nn_grad

ENABLED = False


@contextlib.contextmanager
def enabled():
    global ENABLED
    prev, ENABLED = ENABLED, True
    try:
        yield
    finally:
        ENABLED = prev


def r16(t):
    return t.to(torch.bfloat16).to(t.dtype)


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, padding):
        rx, rw = r16(x), r16(w)
        ctx.save_for_backward(rx, rw)
        ctx.cfg = (stride, padding, x.shape, w.shape, b is not None)
        return F.conv2d(rx, rw, b, stride=stride, padding=padding)

    @staticmethod
    def backward(ctx, dy):
        rx, rw = ctx.saved_tensors
        stride, padding, xs, ws, has_b = ctx.cfg
        rdy = r16(dy)
        dx = nn_grad.conv2d_input(xs, rw, rdy, stride=stride, padding=padding)
        dw = nn_grad.conv2d_weight(rx, ws, rdy, stride=stride, padding=padding)
        db = dy.sum((0, 2, 3)) if has_b else None
        return dx, dw, db, None, None


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        rx, rw = r16(x), r16(w)
        ctx.save_for_backward(rx, rw)
        ctx.has_b = b is not None
        return F.linear(rx, rw, b)

    @staticmethod
    def backward(ctx, dy):
        rx, rw = ctx.saved_tensors
        rdy = r16(dy)
        dx = rdy @ rw
        dw = rdy.reshape(-1, rdy.shape[-1]).t() @ rx.reshape(-1, rx.shape[-1])
        db = dy.reshape(-1, dy.shape[-1]).sum(0) if ctx.has_b else None
        return dx, dw, db


class _Matmul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ra, rb = r16(a), r16(b)
        ctx.save_for_backward(ra, rb)
        return torch.matmul(ra, rb)

    @staticmethod
    def backward(ctx, dy):
        ra, rb = ctx.saved_tensors
        rdy = r16(dy)
        return torch.matmul(rdy, rb.transpose(-2, -1)), torch.matmul(ra.transpose(-2, -1), rdy)


def conv2d(x, w, b=None, stride=1, padding=0, groups=1):
    if not ENABLED or groups != 1:
        return F.conv2d(x, w, b, stride=stride, padding=padding, groups=groups)
    return _Conv.apply(x, w, b, stride, padding)


def linear(x, w, b=None):
    return _Linear.apply(x, w, b) if ENABLED else F.linear(x, w, b)


def matmul(a, b):
    return _Matmul.apply(a, b) if ENABLED else torch.matmul(a, b)
