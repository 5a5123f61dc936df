"""Attention dropout fused into the softmax sweep (mdemi_softmax_fwd_drop16: the bf16 copy of
dropout(P) that P.V reads, kept for dV in the backward).  The fused sweep must reproduce the
standalone dropout sweep it replaces (mdemi_dropout_dev16: same counter-hash mask, same bf16
copy) BIT FOR BIT, and a whole Depthformer v8 train-mode forward + backward with dropout active
must be bit-identical with the fusion on and off (MDEMI_FUSE_DROPOUT), including the attention
calls whose V slice the bf16 loaders cannot stage (the fp32 fallback).
Reference: the attention dropout of model/Depthformer/luna_layer.py:213-215,244-246 and
self_attention.py:72-74 (nn.Dropout, layers.py:8)."""
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
    outputs, attention maps and every parameter gradient equal bit for bit with the attention
    dropout fused (softmax sweep, saved bf16 dropout(P)) and as standalone sweeps."""
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

