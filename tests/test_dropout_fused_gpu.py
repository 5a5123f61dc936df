"""Dropout fused into its producer: the GEMM epilogue (mdemi_gemm_desc.drop_seed) and the
attention softmax sweep (mdemi_softmax_fwd_drop16).  Every fused form must reproduce the
standalone sweep it replaces (mdemi_dropout_dev / _dev16: same counter-hash mask, same fp32
values, same bf16 copy) BIT FOR BIT -- after a forward activation, before an activation-gradient
multiply, through split-K (separate reduce and in-kernel combine), two-level attention batches
and the bf16-operand kernel -- and a whole Depthformer v8 train-mode forward + backward with
dropout active must be bit-identical with the fusion on and off (MDEMI_FUSE_DROPOUT).
Reference: nn.Dropout in model/Depthformer/feed_forward.py:26, luna_layer.py:172-173,213-215,
244-246, self_attention.py:72-74, layers.py:8."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def mf():
    from mdemi import _lib
    from mdemi import functional
    _lib.load()
    return functional


def _sweep(L, t, p, seed, add, off, t16=None):
    L.call("mdemi_dropout_dev16", t.data_ptr(), t.data_ptr(), L.ptr(t16), t.numel(), float(p), seed.data_ptr(), add,
           off, L.stream())


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("split", [1, 4, "inline"])
@pytest.mark.parametrize("act", ["none", "gelu", "silu_grad", "gelu_grad"])
def test_gemm_epilogue_dropout_matches_sweep(mf, prec, split, act):
    from mdemi import _lib as L
    lib = L.load()
    torch.manual_seed(1)
    M, N, K = 1000, 384, 320
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.05
    b = torch.randn(N, device=DEV)
    h = torch.randn(M, N, device=DEV)
    seed = torch.tensor([0x1234_5678_9ABC], dtype=torch.int64, device=DEV)
    p, add, off = 0.3, 7, 1000
    grad = act.endswith("_grad")
    code = {"none": L.ACT_NONE, "gelu": L.ACT_GELU, "silu_grad": L.ACT_SILU_GRAD, "gelu_grad": L.ACT_GELU_GRAD}[act]
    kw = dict(lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, bias=b, bias_mode=L.BIAS_COL,
              split_k=1 if split == 1 else 4)
    if split == "inline":
        assert lib.mdemi_gemm_set_options(1, 1) == 0
    try:
        with mf.matmul_precision(prec):
            ref = torch.empty(M, N, device=DEV)
            ref16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            if grad:  # the dropout backward between the product and the act'(h) multiply
                mf.gemm(x, w, ref, M, N, K, **kw)
                _sweep(L, ref, p, seed, add, off)
                base = {"silu_grad": L.ACT_SILU, "gelu_grad": L.ACT_GELU}[act]
                L.call("mdemi_elementwise", L.EW_ACT_BWD, h.data_ptr(), ref.data_ptr(), ref.data_ptr(), ref.numel(),
                       float(base), 0.0, L.stream())
                L.call("mdemi_cast_bf16", ref.data_ptr(), ref16.data_ptr(), ref.numel(), L.stream())
            else:
                mf.gemm(x, w, ref, M, N, K, act=code, **kw)
                _sweep(L, ref, p, seed, add, off, ref16)
            got = torch.full((M, N), float("nan"), device=DEV)
            got16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            extra = dict(act=code, aux=h if grad else None, ldaux=N if grad else 0, drop=(p, seed, add, off))
            if prec == "bf16":
                mf.gemm(None, None, got, M, N, K, a16=x.to(torch.bfloat16), b16=w.to(torch.bfloat16), c16=got16,
                        **kw, **extra)
            else:
                mf.gemm(x, w, got, M, N, K, **kw, **extra)
                L.call("mdemi_cast_bf16", got.data_ptr(), got16.data_ptr(), got.numel(), L.stream())
        torch.cuda.synchronize()
    finally:
        lib.mdemi_gemm_set_options(1, 0)
    kept = (got != 0).float().mean().item()
    assert 0.6 < kept < 0.8, kept  # the mask is live (p = 0.3)
    assert torch.equal(ref, got), (ref - got).abs().max().item()
    assert torch.equal(ref16, got16)


def test_batched_attention_product_dropout_matches_sweep(mf):
    """dP = dO . V^T over (image, head) pairs (two-level batch, heads as column slices): the
    epilogue mask index is each element's offset in the [B, heads, Sq, Sk] buffer."""
    from mdemi import _lib as L
    torch.manual_seed(2)
    B, heads, Sq, Sk, dv = 2, 4, 300, 96, 32
    dout = torch.randn(B * Sq, heads * dv, device=DEV)
    v = torch.randn(B * Sk, heads * dv, device=DEV)
    seed = torch.tensor([99], dtype=torch.int64, device=DEV)
    hs = Sq * Sk
    kw = dict(lda=heads * dv, ldb=heads * dv, ldc=Sk, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, batch=B * heads,
              a_bstride=Sq * heads * dv, b_bstride=Sk * heads * dv, c_bstride=heads * hs, inner=(heads, dv, dv, hs))
    for prec in ("fp32", "bf16"):
        with mf.matmul_precision(prec):
            ref = torch.empty(B, heads, Sq, Sk, device=DEV)
            got = torch.empty_like(ref)
            mf.gemm(dout, v, ref, Sq, Sk, dv, **kw)
            _sweep(L, ref, 0.1, seed, 0, 0)
            mf.gemm(dout, v, got, Sq, Sk, dv, drop=(0.1, seed, 0, 0), **kw)
        torch.cuda.synchronize()
        assert torch.equal(ref, got), prec


@pytest.mark.parametrize("cols", [96, 300, 2000])
def test_softmax_dropped_bf16_copy_matches_sweep(mf, cols):
    from mdemi import _lib as L
    torch.manual_seed(3)
    rows = 777
    x = torch.randn(rows, cols, device=DEV) * 3
    seed = torch.tensor([4242], dtype=torch.int64, device=DEV)
    y_ref = torch.empty_like(x)
    d_ref = torch.empty_like(x)
    d16_ref = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
    L.call("mdemi_softmax_fwd16", x.data_ptr(), y_ref.data_ptr(), None, rows, cols, 0.7, L.stream())
    L.call("mdemi_dropout_dev16", y_ref.data_ptr(), d_ref.data_ptr(), d16_ref.data_ptr(), y_ref.numel(), 0.2,
           seed.data_ptr(), 3, 11, L.stream())
    y = torch.empty_like(x)
    y16 = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
    L.call("mdemi_softmax_fwd_drop16", x.data_ptr(), y.data_ptr(), y16.data_ptr(), rows, cols, 0.7, 0.2,
           seed.data_ptr(), 3, 11, L.stream())
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)  # the softmax itself is unchanged (the backward's operand)
    assert torch.equal(y16.view(torch.int16), d16_ref.view(torch.int16))
    assert 0.7 < (y16 != 0).float().mean().item() < 0.9


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_depthformer_train_step_fused_dropout_bit_identical(mf, prec):
    """Depthformer v8 in train mode with attention dropout 0.1 and feed-forward dropout 0.2:
    outputs, attention maps and every parameter gradient equal bit for bit with the dropout
    fusion on (GEMM epilogues, softmax sweep, saved bf16 dropout(P)) and off (standalone sweeps)."""
    from mdemi.model.Depthformer import DepthformerV8
    from oracle.weights import closed_form_fill, rng_array
    opt = {"hidden_dim": 64, "num_heads": 4, "num_bins": 64, "num_aux": 32, "img_size": [128, 160],
           "attn_drop_prob": 0.1, "drop_prob": 0.2}
    torch.manual_seed(0)
    m = DepthformerV8.build(opt, 1e-3, 10.0)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    closed_form_fill(sd, seed=0.37, scale=0.03)
    img = torch.from_numpy(rng_array((2, 3, 128, 160), 41)).float().to(DEV)
    dy = torch.from_numpy(rng_array((2, 1, 64, 80), 42)).float().to(DEV)
    m = m.to(DEV).train()

    def run(fuse):
        prev = mf._FUSE_DROP[0]
        mf._FUSE_DROP[0] = fuse
        m.load_state_dict({k: v.to(DEV) for k, v in sd.items()})
        m.zero_grad(set_to_none=True)
        mf._drop_counter[0] = 0
        torch.manual_seed(123)  # the on-device seed draws
        try:
            with mf.matmul_precision(prec):
                depth, centers, attn = m(img)
                (depth * dy).sum().backward()
        finally:
            mf._FUSE_DROP[0] = prev
        torch.cuda.synchronize()
        return [depth.detach().clone(), centers.detach().clone()] + [a.detach().clone() for a in attn], \
            {k: p.grad.detach().clone() for k, p in m.named_parameters()}

    out0, g0 = run(False)
    out1, g1 = run(True)
    for i, (a, b) in enumerate(zip(out0, out1)):
        assert torch.equal(a, b), i
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
    out2, _ = run(True)
    assert torch.equal(out1[0], out2[0])  # deterministic


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("residual", [False, True])
def test_linear_dropout_residual_fused_matches_composite(mf, prec, residual):
    """mf.linear(..., p, training=True) -- dropout (and the residual add) in the projection's
    epilogue, the dropout backward as one sweep -- against dropout(linear(x)) (+ add): output
    and the input / weight / bias / residual gradients bit for bit."""
    torch.manual_seed(4)
    M, K, N = 1200, 256, 192
    x0 = torch.randn(M, K, device=DEV)
    w0 = torch.randn(N, K, device=DEV) * 0.05
    b0 = torch.randn(N, device=DEV)
    r0 = torch.randn(M, N, device=DEV)
    dy = torch.randn(M, N, device=DEV)

    def run(fuse):
        prev = mf._FUSE_DROP[0]
        mf._FUSE_DROP[0] = fuse
        mf._drop_counter[0] = 0
        torch.manual_seed(77)
        x, w, b, r = (t.clone().requires_grad_() for t in (x0, w0, b0, r0))
        try:
            with mf.matmul_precision(prec):
                y = mf.linear(x, w, b, residual=r if residual else None, p=0.2, training=True)
                (y * dy).sum().backward()
        finally:
            mf._FUSE_DROP[0] = prev
        torch.cuda.synchronize()
        return [y.detach(), x.grad, w.grad, b.grad] + ([r.grad] if residual else [])

    ref, got = run(False), run(True)
    assert 0.7 < (got[0] != (r0 if residual else 0)).float().mean().item() <= 1.0
    for i, (a, b) in enumerate(zip(ref, got)):
        assert torch.equal(a, b), i
