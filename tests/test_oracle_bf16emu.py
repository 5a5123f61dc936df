"""The oracle's bf16 mixed-precision emulation (oracle/bf16emu.py), CPU only: outside the
context its ops are torch's; inside, each product takes bf16-rounded operands in the forward
and in both backward products, and a bias gradient sums the unrounded incoming gradient."""
import torch
import torch.nn.functional as F

from oracle import bf16emu as E


def _r(t):
    return t.to(torch.bfloat16).double()


def test_disabled_is_torch():
    g = torch.Generator().manual_seed(0)
    x, w, b = (torch.randn(2, 5, 6, 7, generator=g, dtype=torch.float64), torch.randn(4, 5, 3, 3, generator=g,
               dtype=torch.float64), torch.randn(4, generator=g, dtype=torch.float64))
    assert torch.equal(E.conv2d(x, w, b, padding=1), F.conv2d(x, w, b, padding=1))
    a = torch.randn(3, 8, dtype=torch.float64)
    assert torch.equal(E.linear(a, torch.ones(2, 8, dtype=torch.float64)), F.linear(a, torch.ones(2, 8).double()))


def test_linear_and_matmul_round_every_product():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(7, 9, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(5, 9, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(5, generator=g, dtype=torch.float64, requires_grad=True)
    dy = torch.randn(7, 5, generator=g, dtype=torch.float64)
    with E.enabled():
        y = E.linear(x, w, b)
    y.backward(dy)
    assert torch.allclose(y, _r(x) @ _r(w).t() + b, rtol=0, atol=1e-12)
    assert torch.allclose(x.grad, _r(dy) @ _r(w), rtol=0, atol=1e-12)
    assert torch.allclose(w.grad, _r(dy).t() @ _r(x), rtol=0, atol=1e-12)
    assert torch.allclose(b.grad, dy.sum(0), rtol=0, atol=1e-12)
    a = torch.randn(2, 3, 4, 6, generator=g, dtype=torch.float64, requires_grad=True)
    c = torch.randn(2, 3, 6, 5, generator=g, dtype=torch.float64, requires_grad=True)
    d = torch.randn(2, 3, 4, 5, generator=g, dtype=torch.float64)
    with E.enabled():
        z = E.matmul(a, c)
    z.backward(d)
    assert torch.allclose(z, _r(a) @ _r(c), rtol=0, atol=1e-12)
    assert torch.allclose(a.grad, _r(d) @ _r(c).transpose(-1, -2), rtol=0, atol=1e-12)
    assert torch.allclose(c.grad, _r(a).transpose(-1, -2) @ _r(d), rtol=0, atol=1e-12)


def test_conv_rounds_groups1_only():
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, 4, 9, 8, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(6, 4, 3, 3, generator=g, dtype=torch.float64, requires_grad=True)
    with E.enabled():
        y = E.conv2d(x, w, None, stride=2, padding=1)
        dw = torch.randn(4, 1, 3, 3, generator=g, dtype=torch.float64)
        yd = E.conv2d(x.detach(), dw, None, padding=1, groups=4)
    assert torch.equal(yd, F.conv2d(x.detach(), dw, None, padding=1, groups=4))  # depthwise: fp32 on the GPU too
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(dy)
    xr = _r(x.detach()).requires_grad_()
    wr = _r(w.detach()).requires_grad_()
    yr = F.conv2d(xr, wr, None, stride=2, padding=1)
    yr.backward(_r(dy))
    assert torch.allclose(y, yr, rtol=0, atol=1e-12)
    assert torch.allclose(x.grad, xr.grad, rtol=0, atol=1e-12)
    assert torch.allclose(w.grad, wr.grad, rtol=0, atol=1e-12)
