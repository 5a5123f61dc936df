"""fp32 GEMM on the bf16 matrix cores (precision "fp32e", mdemi_gemm_f32e).

Each fp32 operand is split exactly into three bf16 planes and six plane products are
accumulated in fp32.  The claim is that this IS an fp32 GEMM: its error against the
fp64 product of the same fp32 operands is no larger than that of the exact-product fp32
MFMA kernel (precision "fp32").  Tolerance, per output tensor:

    max|C_f32e - C_64| <= 2 * max|C_f32 - C_64| + 2^-24 * max_ij sum_k |a_ik||b_kj|

on every operand layout the model uses (Linear fwd / dgrad / wgrad with the bias-gradient
row sums, GELU applied on load, deep split-K, implicit-im2col conv fwd / dgrad / wgrad
with zero and replicate padding)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
EPS24 = 2.0 ** -24


@pytest.fixture(scope="module")
def mf():
    from mdemi import _lib
    from mdemi import functional
    _lib.load()
    return functional


def _errs(results, ref, absprod):
    """max |err| of each precision's result against the fp64 reference."""
    return {k: (v.double().cpu() - ref).abs().max().item() for k, v in results.items()}, absprod.max().item()


def _check(what, results, ref, absprod):
    e, scale = _errs(results, ref, absprod)
    lim = 2.0 * e["fp32"] + EPS24 * scale
    assert e["fp32e"] <= lim, (what, e, lim)
    return e


@pytest.mark.parametrize("M,N,K,gelu", [(300, 200, 96, False), (1000, 384, 1536, True), (64, 96, 40000, False),
                                        (4096, 768, 3072, True)])
def test_linear_f32e_matches_fp32_accuracy(mf, M, N, K, gelu):
    torch.manual_seed(0)
    x0 = torch.randn(M, K, device=DEV)
    w0 = torch.randn(N, K, device=DEV) * K ** -0.5
    b0 = torch.randn(N, device=DEV)
    dy = torch.randn(M, N, device=DEV)
    out = {}
    for prec in ("fp32", "fp32e"):
        x = x0.clone().requires_grad_()
        w = w0.clone().requires_grad_()
        b = b0.clone().requires_grad_()
        with mf.matmul_precision(prec):
            y = mf.linear(x, w, b, in_gelu=gelu)
            y.backward(dy)
        torch.cuda.synchronize()
        out[prec] = (y.detach(), x.grad, w.grad, b.grad)
    xd, wd, dyd = x0.double().cpu(), w0.double().cpu(), dy.double().cpu()
    xg = torch.nn.functional.gelu(xd) if gelu else xd
    ref = xg @ wd.T + b0.double().cpu()
    _check("fwd", {k: v[0] for k, v in out.items()}, ref, xg.abs() @ wd.abs().T)
    gx = dyd @ wd
    if gelu:  # d gelu(x)/dx applied to the product (the dgrad epilogue)
        xr = xd.clone().requires_grad_()
        torch.nn.functional.gelu(xr).backward(gx)
        gx = xr.grad
        absg = (dyd.abs() @ wd.abs()) * 1.2
    else:
        absg = dyd.abs() @ wd.abs()
    _check("dgrad", {k: v[1] for k, v in out.items()}, gx, absg)
    _check("wgrad", {k: v[2] for k, v in out.items()}, dyd.T @ xg, dyd.abs().T @ xg.abs())
    _check("bias grad", {k: v[3] for k, v in out.items()}, dyd.sum(0), dyd.abs().sum(0))


@pytest.mark.parametrize("cin,cout,k,stride,pad,hw,replicate",
                         [(64, 96, 3, 1, 1, (17, 23), False), (128, 64, 1, 1, 0, (30, 40), False),
                          (36, 48, 3, 1, 1, (19, 26), False), (64, 64, 3, 1, 1, (15, 20), True),
                          (512, 256, 3, 1, 1, (44, 152), False)])
def test_conv_f32e_matches_fp32_accuracy(mf, cin, cout, k, stride, pad, hw, replicate):
    from mdemi import _lib as L
    torch.manual_seed(2)
    x0 = torch.randn(2, *hw, cin, device=DEV)  # NHWC
    w0 = torch.randn(cout, cin, k, k, device=DEV) * (cin * k * k) ** -0.5
    out = {}
    dy = None
    for prec in ("fp32", "fp32e"):
        x = x0.clone().requires_grad_()
        w = w0.clone().requires_grad_()
        with mf.matmul_precision(prec):
            y = mf.conv2d_nhwc(x, w, None, stride=stride, pad=pad,
                               pad_mode=L.PAD_REPLICATE if replicate else L.PAD_ZERO)
            if dy is None:
                dy = torch.randn_like(y)
            y.backward(dy)
        torch.cuda.synchronize()
        out[prec] = (y.detach().permute(0, 3, 1, 2), x.grad.permute(0, 3, 1, 2), w.grad)
    F = torch.nn.functional

    def conv(a, b):
        if replicate:
            a = F.pad(a, (pad, pad, pad, pad), mode="replicate")
            return F.conv2d(a, b, stride=stride)
        return F.conv2d(a, b, stride=stride, padding=pad)

    xc = x0.cpu().permute(0, 3, 1, 2).double()
    wc, dyc = w0.cpu().double(), dy.cpu().permute(0, 3, 1, 2).double()
    _check("conv fwd", {k_: v[0] for k_, v in out.items()}, conv(xc, wc), conv(xc.abs(), wc.abs()))
    xr, wr = xc.clone().requires_grad_(), wc.clone().requires_grad_()
    conv(xr, wr).backward(dyc)
    xa, wa = xc.abs().requires_grad_(), wc.abs().requires_grad_()
    conv(xa, wa).backward(dyc.abs())
    _check("conv dgrad", {k_: v[1] for k_, v in out.items()}, xr.grad, xa.grad)
    _check("conv wgrad", {k_: v[2] for k_, v in out.items()}, wr.grad, wa.grad)


def test_f32e_variants_bit_identical(mf):
    """Every 16-bit-family variant (LDS buffering, 128- / 256-row tiles) adds the same
    products in the same order."""
    from mdemi import _lib as L
    lib = L.load()
    torch.manual_seed(5)
    x = torch.randn(2000, 640, device=DEV)
    w = torch.randn(384, 640, device=DEV)
    outs = []
    try:
        for v in (0, 1, 2):
            assert lib.mdemi_gemm_set_variant_m16(v) == 0
            with mf.matmul_precision("fp32e"):
                outs.append(mf.linear(x, w).clone())
    finally:
        lib.mdemi_gemm_set_variant_m16(-1)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
