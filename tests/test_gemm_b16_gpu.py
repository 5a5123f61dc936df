"""bf16-operand GEMM (csrc/gemm_b16_kernel.h, mdemi_gemm_bf16x): operands stored in bf16
and DMA'd straight into LDS.  For operands that are the RNE bf16 of fp32 tensors, every
result must be BIT-IDENTICAL to the bf16 GEMM on the fp32 tensors (mdemi_gemm_bf16, which
rounds the same values as it stages them) -- on every layout pair the model uses (dense
k-/m,n-contiguous, implicit-im2col forward / data gradient / weight gradient, zero and
replicate padding), batched and two-level-batched products, split K and the tail split,
ragged edges, every fused epilogue, both tile variants -- and the optional bf16 output copy
must equal the RNE bf16 of the fp32 output.  Layouts the DMA loaders cannot stage fall back
to the fp32-operand kernel.  Reference: the autocast bf16 conv / linear / bmm of
model/Depthformer/layer_utils.py:6-34, luna_layer.py:181-259 (BASELINE configs[4])."""
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


def _b(t):
    return t.to(torch.bfloat16)


def _run(mf, L, fp, bf, C_shape, variant, **kw):
    """C from the fp32-operand bf16 GEMM and from the bf16-operand one (forced variant)."""
    lib = L.load()
    A, B = fp
    A16, B16 = bf
    ref = torch.full(C_shape, float("nan"), device=DEV)
    got = torch.full(C_shape, float("nan"), device=DEV)
    c16 = torch.empty(C_shape, device=DEV, dtype=torch.bfloat16)
    with mf.matmul_precision("bf16"):
        mf.gemm(A, B, ref, **kw)
        assert lib.mdemi_gemm_set_variant_b16(variant) == 0
        try:
            mf.gemm(None, None, got, a16=A16, b16=B16, c16=c16, **kw)
        finally:
            lib.mdemi_gemm_set_variant_b16(-1)
    torch.cuda.synchronize()
    return ref, got, c16


def _check(ref, got, c16, what):
    assert torch.equal(ref, got), (what, (ref - got).abs().max().item())
    assert torch.equal(c16, ref.to(torch.bfloat16)), what


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(3000, 384, 640), (1000, 200, 136), (4736, 1024, 256), (64, 96, 40000)])
def test_dense_layouts_bit_identical(mf, variant, M, N, K):
    from mdemi import _lib as L
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.05
    bias = torch.randn(N, device=DEV)
    dy = torch.randn(M, N, device=DEV)
    res = torch.randn(M, N, device=DEV)
    x, w, dy = (_b(t).float() for t in (x, w, dy))  # exactly representable: the bf16 copies are exact
    # forward: Y = X W^T + b, SiLU, + residual  (KCONTIG x KCONTIG)
    ref, got, c16 = _run(mf, L, (x, w), (_b(x), _b(w)), (M, N), variant, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                         a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, bias=bias, bias_mode=L.BIAS_COL,
                         act=L.ACT_SILU, residual=res, ldres=N, split_k=1)
    _check(ref, got, c16, "fwd")
    # data gradient: dX = dY W  (KCONTIG x MNCONTIG)
    ref, got, c16 = _run(mf, L, (dy, w), (_b(dy), _b(w)), (M, K), variant, M=M, N=K, K=N, lda=N, ldb=K, ldc=K,
                         a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG)
    _check(ref, got, c16, "dgrad")
    # weight gradient: dW = dY^T X  (MNCONTIG x MNCONTIG), split K over the M rows
    ref, got, c16 = _run(mf, L, (dy, x), (_b(dy), _b(x)), (N, K), variant, M=N, N=K, K=M, lda=N, ldb=K, ldc=K,
                         a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG, split_k=max(1, M // 512))
    _check(ref, got, c16, "wgrad")
    # m-contiguous A with k-contiguous B (MNCONTIG x KCONTIG): X^T-style product
    ref, got, c16 = _run(mf, L, (x, dy), (_b(x), _b(dy)), (K, N), variant, M=K, N=N, K=M, lda=K, ldb=M, ldc=N,
                         a_layout=L.L_MNCONTIG, b_layout=L.L_KCONTIG)
    _check(ref, got, c16, "mn x kc")


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("cin,cout,k,pad,hw,mode", [(64, 96, 3, 1, (17, 23), "zero"), (128, 64, 3, 1, (30, 40), "rep"),
                                                    (32, 40, 5, 2, (9, 12), "zero"), (256, 256, 3, 1, (60, 80), "zero")])
def test_conv_layouts_bit_identical(mf, variant, cin, cout, k, pad, hw, mode):
    from mdemi import _lib as L
    torch.manual_seed(1)
    n = 2
    h, w = hw
    pm = L.PAD_REPLICATE if mode == "rep" else L.PAD_ZERO
    x = _b(torch.randn(n, h, w, cin, device=DEV)).float()
    wt = _b(torch.randn(cout, k * k * cin, device=DEV) * 0.05).float()  # (ky,kx,c)-ordered rows
    dy = _b(torch.randn(n, h, w, cout, device=DEV)).float()
    M, K = n * h * w, k * k * cin
    g = mf._geom(n, h, w, cin, h, w, k, k, 1, pad, pm)
    ref, got, c16 = _run(mf, L, (x, wt), (_b(x), _b(wt)), (n, h, w, cout), variant, M=M, N=cout, K=K, lda=0, ldb=K,
                         ldc=cout, a_layout=L.L_CONV, b_layout=L.L_KCONTIG, conv=g)
    _check(ref, got, c16, "conv fwd")
    # weight gradient: dW[co][(ky,kx,c)] = sum_pixels dY[p][co] x im2col(X)[p][(ky,kx,c)]
    ref, got, c16 = _run(mf, L, (dy, x), (_b(dy), _b(x)), (cout, K), variant, M=cout, N=K, K=M, lda=cout, ldb=0,
                         ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_CONV, conv=g, split_k=max(1, M // 1024))
    _check(ref, got, c16, "conv wgrad")
    if mode == "zero":  # data gradient: dX = conv(dY, flip(W)^T) with pad k-1-p (wd [(ky,kx,co)][c])
        wd = _b(torch.randn(k * k * cout, cin, device=DEV) * 0.05).float()
        gd = mf._geom(n, h, w, cout, h, w, k, k, 1, k - 1 - pad, L.PAD_ZERO)
        ref, got, c16 = _run(mf, L, (dy, wd), (_b(dy), _b(wd)), (n, h, w, cin), variant, M=M, N=cin, K=k * k * cout,
                             lda=0, ldb=cin, ldc=cin, a_layout=L.L_CONV, b_layout=L.L_MNCONTIG, conv=gd)
        _check(ref, got, c16, "conv dgrad")


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_batched_attention_products_bit_identical(mf, variant):
    """Two-level batch (image, head) as the Luna / self-attention products issue them:
    scores = Q K^T (k-contiguous both), out = P V (V m/n-contiguous)."""
    from mdemi import _lib as L
    torch.manual_seed(2)
    b, heads, S, T, d = 2, 4, 1200, 256, 64
    q = _b(torch.randn(b, S, heads * d, device=DEV)).float()
    kk = _b(torch.randn(b, T, heads * d, device=DEV)).float()
    p = _b(torch.rand(b * heads, S, T, device=DEV)).float()
    inner = (heads, d, d, S * T)
    ref, got, c16 = _run(mf, L, (q, kk), (_b(q), _b(kk)), (b * heads, S, T), variant, M=S, N=T, K=d, lda=heads * d,
                         ldb=heads * d, ldc=T, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, batch=b * heads,
                         a_bstride=S * heads * d, b_bstride=T * heads * d, c_bstride=heads * S * T, inner=inner)
    _check(ref, got, c16, "scores")
    inner2 = (heads, S * T, d, d)
    ref, got, c16 = _run(mf, L, (p, kk), (_b(p), _b(kk)), (b, S, heads * d), variant, M=S, N=d, K=T, lda=T,
                         ldb=heads * d, ldc=heads * d, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG, batch=b * heads,
                         a_bstride=heads * S * T, b_bstride=T * heads * d, c_bstride=S * heads * d, inner=inner2)
    _check(ref, got, c16, "p v")


def test_unstageable_layout_falls_back(mf):
    """K % 8 != 0 (a k-contiguous 16-B chunk would straddle the K edge): the fp32 operands are
    used (same products), and without them the call refuses rather than guess."""
    from mdemi import _lib as L
    lib = L.load()
    torch.manual_seed(3)
    M, N, K = 300, 200, 100
    x = _b(torch.randn(M, K, device=DEV)).float()
    w = _b(torch.randn(N, K, device=DEV)).float()
    d = L.GemmDesc()
    d.M, d.N, d.K, d.batch, d.lda, d.ldb, d.ldc = M, N, K, 1, K, K, N
    d.a_layout = d.b_layout = L.L_KCONTIG
    d.split_k = 1
    assert lib.mdemi_gemm_bf16x_supported(d, _b(x).data_ptr(), _b(w).data_ptr()) == 0
    ref = torch.empty(M, N, device=DEV)
    got = torch.empty(M, N, device=DEV)
    c16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    with mf.matmul_precision("bf16"):
        mf.gemm(x, w, ref, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG)
        mf.gemm(x, w, got, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
                a16=_b(x), b16=_b(w), c16=c16)
        with pytest.raises(RuntimeError, match="no bf16 path"):
            mf.gemm(None, None, got, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
                    a16=_b(x), b16=_b(w))
    torch.cuda.synchronize()
    _check(ref, got, c16, "fallback")


@pytest.mark.parametrize("bn", ["train", "eval"])
def test_bf16_storage_step_matches_fp32_operand_step(mf, bn):
    """The bf16 storage path (every bf16 GEMM on bf16 copies: producer-written or one cast per
    tensor, reused by the later GEMMs on it) against the same Depthformer v8 forward + backward
    with every operand fp32 (set_bf16_storage(False)): outputs, attention maps and every
    gradient bit-identical, except the conv / linear bias gradients, which the storage path sums
    from the same unrounded fp32 dY in a column-sum sweep instead of inside the GEMM (fp32
    reassociation only)."""
    from mdemi.model.Depthformer import DepthformerV8
    from oracle.weights import closed_form_fill, rng_array
    opt = {"hidden_dim": 64, "num_heads": 4, "num_bins": 64, "num_aux": 32, "img_size": [128, 160],
           "attn_drop_prob": 0.0, "drop_prob": 0.0}
    torch.manual_seed(0)
    m = DepthformerV8.build(opt, 1e-3, 10.0)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    closed_form_fill(sd, seed=0.61, scale=0.03)
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    if bn == "eval":
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.eval()
    img = torch.from_numpy(rng_array((2, 3, 128, 160), 31)).float().to(DEV)
    dy = torch.from_numpy(rng_array((2, 1, 64, 80), 32)).float().to(DEV)

    def run(storage):
        prev = mf.get_bf16_storage()
        mf.set_bf16_storage(storage)
        m.load_state_dict({k: v.to(DEV) for k, v in sd.items()})
        m.zero_grad(set_to_none=True)
        try:
            with mf.matmul_precision("bf16"):
                depth, centers, attn = m(img)
                (depth * dy).sum().backward()
        finally:
            mf.set_bf16_storage(prev)
        torch.cuda.synchronize()
        return [depth.detach().clone(), centers.detach().clone()] + [a.detach().clone() for a in attn], \
            {k: p.grad.detach().clone() for k, p in m.named_parameters()}

    out0, g0 = run(False)
    out1, g1 = run(True)
    for i, (a, b) in enumerate(zip(out0, out1)):
        assert torch.equal(a, b), i
    n_bias, worst = 0, (0.0, None)
    for k in g0:
        if k.endswith(".bias") and not torch.equal(g0[k], g1[k]):
            n_bias += 1
            import bf16_criterion as crit
            sh = crit.SHIFT_INVARIANT.search(k)
            if sh:  # exact gradient zero (softmax shift invariance): both are residue, held in size
                vb = k[:sh.start()] + crit._VALUE_OF[sh.group(1)] + ".bias"
                lim = 1e-4 * g0[vb].abs().max().item()
                assert g0[k].abs().max().item() <= lim and g1[k].abs().max().item() <= lim, k
            else:  # fp32 reassociation of a sum over every pixel: relative L2 within 1e-4
                rel = ((g1[k] - g0[k]).norm() / g0[k].norm().clamp_min(1e-30)).item()
                worst = max(worst, (rel, k))
                assert rel <= 1e-4, (k, rel)
        else:
            assert torch.equal(g0[k], g1[k]), k
    print(f"bf16 storage step == fp32-operand bf16 step bit for bit; {n_bias} bias gradients reassociated "
          f"(worst relative L2 {worst})")


def test_adamw_maintains_bf16_weight_copies(mf):
    """Under bf16 storage FusedAdamW writes each GEMM weight's bf16 copy in the update
    (mdemi_adamw_step16): after a step every maintained copy equals the RNE cast of the new
    weights bit for bit and is the valid recorded copy, and the next forward casts no
    parameter (only activations without a producer-written copy are cast)."""
    from mdemi import _lib as L
    from mdemi.model.Depthformer import DepthformerV8
    from mdemi.train.optim import FusedAdamW
    from oracle.weights import closed_form_fill, rng_array
    opt = {"hidden_dim": 64, "num_heads": 4, "num_bins": 64, "num_aux": 32, "img_size": [128, 160],
           "attn_drop_prob": 0.0, "drop_prob": 0.0}
    torch.manual_seed(0)
    m = DepthformerV8.build(opt, 1e-3, 10.0)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    closed_form_fill(sd, seed=0.61, scale=0.03)
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    img = torch.from_numpy(rng_array((2, 3, 128, 160), 31)).float().to(DEV)
    dy = torch.from_numpy(rng_array((2, 1, 64, 80), 32)).float().to(DEV)
    o = FusedAdamW(m.parameters(), lr=1e-4, weight_decay=1e-2, max_grad_norm=0.1)
    ptrs = {p.data_ptr() for p in m.parameters()}
    casts = []
    real_call = L.call

    def counting(name, *args):
        if name == "mdemi_cast_bf16" and args[0] in ptrs:
            casts.append(args[0])
        return real_call(name, *args)

    prev = mf.get_bf16_storage()
    mf.set_bf16_storage(True)
    try:
        with mf.matmul_precision("bf16"):
            for it in range(3):
                casts.clear()
                L.call = counting
                try:
                    depth, _, _ = m(img)
                finally:
                    L.call = real_call
                (depth * dy).sum().backward()
                o.step()
                o.zero_grad()
                if it == 0:
                    n_first = len(casts)
                else:
                    assert not casts, (it, len(casts))
                torch.cuda.synchronize()
                assert o._b16, "no parameter got a maintained bf16 copy"
                for p, b in o._b16.items():
                    assert torch.equal(b, p.detach().to(torch.bfloat16))
                    assert mf.b16_of(p, convert=False) is b
    finally:
        mf.set_bf16_storage(prev)
    print(f"{len(o._b16)} weights kept in bf16 by the update; first forward cast {n_first}, later ones 0")
