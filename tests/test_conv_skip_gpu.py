"""EfficientNet InvertedResidual blocks route their skip through conv_pw (mf.conv2d_nhwc_skip):
the block input's two gradients (through the block and through the residual) meet in the
pointwise input-gradient GEMM's epilogue instead of an autograd add.  The step must be
bit-identical with the fusion on and off (MDEMI_CONV_SKIP), in fp32 and under bf16 storage.
Reference: the gen-efficientnet InvertedResidual the reference's encoders load
(model/Adabins/unet_adaptive_bins.py:126-139, model/Depthformer/depthformer_v8.py:84-95)."""
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


def test_pointwise_skip_matches_add(mf):
    torch.manual_seed(5)
    x0 = torch.randn(2, 30, 40, 64, device=DEV)
    w0 = torch.randn(96, 64, 1, 1, device=DEV) * 0.1
    dy = torch.randn(2, 30, 40, 96, device=DEV)
    dr = torch.randn(2, 30, 40, 64, device=DEV)

    def run(fuse):
        prev = mf._FUSE_SKIP[0]
        mf._FUSE_SKIP[0] = fuse
        x, w = x0.clone().requires_grad_(), w0.clone().requires_grad_()
        try:
            y, skip = mf.conv2d_nhwc_skip(x, w)
            ((y * dy).sum() + (skip * dr).sum()).backward()
        finally:
            mf._FUSE_SKIP[0] = prev
        torch.cuda.synchronize()
        return y.detach(), x.grad, w.grad

    for a, b in zip(run(False), run(True)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_efficientnet_step_with_conv_skip_bit_identical(mf, prec):
    from mdemi.model.Adabins import UnetAdaptiveBins
    from oracle.weights import closed_form_fill, rng_array
    torch.manual_seed(0)
    m = UnetAdaptiveBins.build(32, 1e-3, 10.0)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    closed_form_fill(sd, seed=0.29, scale=0.03)
    img = torch.from_numpy(rng_array((2, 3, 352, 480), 51)).float().to(DEV)  # >= 129 mViT tokens
    m = m.to(DEV).train()

    def run(fuse):
        prev = mf._FUSE_SKIP[0]
        mf._FUSE_SKIP[0] = fuse
        m.load_state_dict({k: v.to(DEV) for k, v in sd.items()})
        m.zero_grad(set_to_none=True)
        mf._drop_counter[0] = 0
        torch.manual_seed(9)
        try:
            with mf.matmul_precision(prec):
                pred, edges = m(img)
                (pred.square().mean() + edges.sum()).backward()
        finally:
            mf._FUSE_SKIP[0] = prev
        torch.cuda.synchronize()
        return [edges.detach().clone(), pred.detach().clone()], \
            {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}

    o0, g0 = run(False)
    o1, g1 = run(True)
    for a, b in zip(o0, o1):
        assert torch.equal(a, b)
    assert g0.keys() == g1.keys() and len(g0) > 100
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
