"""Gradient parity at the benchmark shapes.

The module- and toy-size model tests (test_models_gpu.py) never reach the GEMM paths the
benchmark steps take: deep split-K weight gradients over ~10^5-10^6 pixels, the per-shape
autotuned pipelining variants at the Swin stage-3/4 and DecoderBN shapes, K = 2224 convs.
Here one full train-step backward of each model family runs at its BASELINE resolution
and every parameter gradient is held to the fp64 CPU oracle (oracle/, pinned to the
reference by tests/golden/):

    max|g_gpu - g_64| <= 20 x max|g_cpu32 - g_64| + 1e-3 x max|g_64|

per parameter (the 1e-3 gradient basis of test_models_gpu.py; 20 x the fp32 CPU oracle's
own error covers gradients that are pure rounding noise in exact arithmetic, e.g. biases
feeding a BatchNorm).  Forward outputs: 1e-4 relative (north_star's depth bar), or 20 x
the fp32 oracle's error for the restated EfficientNet-B5 models (ill-conditioned BatchNorm
stacks, see test_models_gpu._check_fwd_conditioned).

The AdaBins and Depthformer tests run under the process's default matmul precision
(MDEMI_MATMUL_PRECISION, "fp32" unless set); the KITTI test checks both fp32 modes.
Under MDEMI_MATMUL_PRECISION=fp32e the Depthformer test misses the fp32 bar on one
cancelling LayerNorm-bias gradient, as the KITTI test documents for large07
(profiles/round2/fp32e8_suite.txt)."""
import pytest
import torch

from test_models_gpu import DEV, _check_fwd_conditioned, _check_param_grads, _filled_state, _no_dropout

pytestmark = pytest.mark.gpu


def test_large07_kitti_train_step_gradients():
    """NeW-CRFs Swin-L (large07) at KITTI 352x1216 (BASELINE configs[2]), batch 1, vs the
    fp64 oracle (computed once), in both fp32 matmul precisions:
    * "fp32" (exact-product fp32 MFMA, the benchmark's): depth within 1e-4 relative and
      every parameter gradient within 20x the fp32 CPU error + 1e-3 of its magnitude;
    * "fp32e" (opt-in, three bf16 planes on the bf16 matrix cores): depth within 1e-4 and
      every gradient within 2e-2 of its magnitude -- its cancelling LayerNorm-bias sums
      miss the fp32 bar (up to 1.03e-2 relative measured, profiles/round2/fp32e_parity_tests.txt),
      so this bounds the opt-in mode's error profile rather than claiming fp32's."""
    from mdemi import functional as mf
    from mdemi.model.NewCRFs import NewCRFDepth
    from oracle import newcrfs as onc
    from oracle.weights import rng_array
    from test_models_gpu import _oracle_run

    torch.set_num_threads(16)
    H, W = 352, 1216
    m = NewCRFDepth(version="large07", max_depth=80.0, drop_path_rate=0.0)
    sd = _filled_state(m, 0.13, 0.02)
    m = m.to(DEV).train()
    img = torch.from_numpy(rng_array((1, 3, H, W), 33))
    dy = torch.from_numpy(rng_array((1, 1, H, W), 34))

    def loss_fn(P):
        dt = next(v.dtype for v in P.values() if torch.is_floating_point(v))
        d = onc.newcrf_depth(P, img.to(dt), "large07", max_depth=80.0)
        (d * dy.to(dt)).sum().backward()
        return d.detach()

    P64, ref = _oracle_run(sd, torch.float64, loss_fn)
    P32, _ = _oracle_run(sd, torch.float32, loss_fn)
    for prec in ("fp32", "fp32e"):
        m.zero_grad(set_to_none=True)
        with mf.matmul_precision(prec):
            depth = m(img.float().to(DEV))
            (depth * dy.float().to(DEV)).sum().backward()
        torch.cuda.synchronize()
        err = (depth.detach().double().cpu() - ref).abs().max().item()
        assert err <= 1e-4 * ref.abs().max().item(), (prec, err)
        n = 0
        for k, p in m.named_parameters():
            r64, r32 = P64[k].grad, P32[k].grad
            e_gpu = (p.grad.double().cpu() - r64).abs().max().item()
            e_cpu = (r32.double() - r64).abs().max().item()
            mag = r64.abs().max().item()
            lim = 20.0 * e_cpu + 1e-3 * mag + 1e-9 if prec == "fp32" else 2e-2 * mag + 1e-9
            assert e_gpu <= lim, (prec, k, e_gpu, e_cpu, mag)
            n += 1
        assert n == len(list(m.parameters()))


def test_adabins_nyu_480x640_train_step_gradients():
    """AdaBins-B5 at NYU 480x640 (BASELINE configs[1] resolution), batch 2.

    End to end: prediction, bin edges and every encoder gradient vs the oracle.  The head
    (DecoderBN, mViT, folded conv_out + bin head) is then checked at the same size on
    seeded NHWC features of the encoder's shapes (the oracle gets the same fp32 values in
    fp64).  Not on the restated B5's own features: at closed-form random weights several
    up1 BatchNorm channels sit at the LeakyReLU kink (near-constant channels, beta ~ 0), so
    which pixels take slope 1 or 0.01 flips with any fp32 forward rounding and those
    channels' bias gradients are discontinuous in the inputs (tools/diag_head.py ... enc:
    one of 97 gradients, up1._net.4.bias, lands at 1.8x the bound in exact-fp32 mode and
    inside it in fp32e mode; on seeded features every gradient is within 0.34x of it).
    The head gets its own closed-form fill: with the full model's fill filtered to the head,
    the mViT's layer-0 feed-forward weight/bias gradients land 41-52x over the bar (27 %
    relative) while every other head gradient passes -- identically with the library of
    this round's start and today's (profiles/round2/diag_adabins_head_*), so it is not a
    regression of this round's kernels.  tools/diag_relu_kink.py finds the cause: one of
    the layer's 614,400 pre-activations is 1.5e-6 in fp64 and lands on the other side of
    the ReLU kink in the GPU's fp32 forward (whose error there is 3.6e-5 of max|z|, 75
    values lie below it), which moves that column's bias gradient by a whole dA element
    (profiles/round2/diag_relu_kink_mvit_layer0.txt): a discontinuity, not an error."""
    from mdemi.model.Adabins import UnetAdaptiveBins
    from oracle import adabins as oab
    from oracle.weights import rng_array
    from test_models_gpu import fake_backend, nhwc_to_nchw

    torch.set_num_threads(16)
    m = UnetAdaptiveBins.build(256, 1e-3, 10.0)
    sd = _filled_state(m, 0.43, 0.03)
    _no_dropout(m)
    m = m.to(DEV).train()
    img = torch.from_numpy(rng_array((2, 3, 480, 640), 82))
    pred, edges = m(img.float().to(DEV))
    (pr, er), (pr32, er32) = (
        _fwd(sd, dt, lambda P, dt: oab.unet_adaptive_bins(P, img.to(dt), 1e-3, 10.0)) for dt in (torch.float64,
                                                                                                 torch.float32))
    _check_fwd_conditioned("pred", pred, pr, pr32)
    _check_fwd_conditioned("bin_edges", edges, er, er32)
    dy = torch.from_numpy(rng_array(tuple(pr.shape), 83))
    (pred * dy.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()

    def loss_fn(P):
        p, _ = oab.unet_adaptive_bins(P, img.to(P["conv_out.0.weight"].dtype), 1e-3, 10.0)
        (p * dy.to(p.dtype)).sum().backward()

    n_enc = sum(1 for k, _ in m.named_parameters() if k.startswith("encoder."))
    assert _check_param_grads(m, sd, loss_fn, rel=1e-3, only="encoder.") == n_enc

    # the head at full size on seeded features of the encoder's shapes (channels, stride)
    chans = {4: (24, 2), 5: (40, 4), 6: (64, 8), 8: (176, 16), 11: (2048, 32)}
    feats = {k: torch.from_numpy(rng_array((2, 480 // st, 640 // st, c), 90 + k)).float().to(DEV)
             for k, (c, st) in chans.items()}
    keys = tuple(chans)
    holder = {}
    head = UnetAdaptiveBins(fake_backend(holder), n_bins=256, min_val=1e-3, max_val=10.0)
    hsd = _filled_state(head, 0.43, 0.03)  # the head's own closed-form fill (see the docstring)
    _no_dropout(head)
    head = head.to(DEV).train()
    ins = {k: feats[k].detach().clone().requires_grad_(True) for k in keys}
    holder.update(ins)
    hp, _ = head(torch.zeros(2, 3, 8, 8, device=DEV))
    (hp * dy.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()

    def head_oracle(dtype):
        P = {k: (v.detach().to(dtype).clone().requires_grad_(True) if torch.is_floating_point(v) else v)
             for k, v in hsd.items()}
        fi = {k: nhwc_to_nchw(ins[k].detach()).cpu().to(dtype).requires_grad_(True) for k in keys}
        p, _ = oab.adabins_head(P, fi, 1e-3, 10.0)
        (p * dy.to(dtype)).sum().backward()
        return P, fi, p.detach()

    P64, F64, p64 = head_oracle(torch.float64)
    P32, F32, _ = head_oracle(torch.float32)
    e = (hp.detach().double().cpu() - p64).abs().max().item()
    assert e <= 1e-4 * p64.abs().max().item(), e
    pairs = [(k, p.grad, P64[k].grad, P32[k].grad) for k, p in head.named_parameters()]
    pairs += [(f"feature {k}", nhwc_to_nchw(ins[k].grad), F64[k].grad, F32[k].grad) for k in keys]
    for k, got, r64, r32 in pairs:
        e_gpu = (got.double().cpu() - r64).abs().max().item()
        e_cpu = (r32.double() - r64).abs().max().item()
        mag = r64.abs().max().item()
        assert e_gpu <= 20.0 * e_cpu + 1e-3 * mag + 1e-9, (k, e_gpu, e_cpu, mag)
    assert len(pairs) == len(list(head.parameters())) + len(keys)


def test_depthformer_v8_nyu_480x640_train_step_gradients():
    """Depthformer v8 at NYU 480x640 with the benchmark's decoder width (hidden 256, 4 heads,
    256 bins, 256 aux tokens), batch 2: depth, centres, the 8 attention maps and every
    parameter gradient vs the oracle."""
    from mdemi.model.Depthformer import DepthformerV8
    from oracle import depthformer as odf
    from oracle.weights import rng_array

    torch.set_num_threads(16)
    opt = {"hidden_dim": 256, "num_heads": 4, "num_bins": 256, "num_aux": 256, "img_size": [480, 640],
           "attn_drop_prob": 0.0, "drop_prob": 0.0}
    m = DepthformerV8.build(opt, 1e-3, 10.0)
    sd = _filled_state(m, 0.53, 0.03)
    m = m.to(DEV).train()
    img = torch.from_numpy(rng_array((2, 3, 480, 640), 84))
    depth, centers, attn = m(img.float().to(DEV))
    (dr, cr, ar), (dr32, cr32, ar32) = (
        _fwd(sd, dt, lambda P, dt: odf.depthformer_v8_full(P, img.to(dt), opt, 1e-3, 10.0))
        for dt in (torch.float64, torch.float32))
    for i, (a, r, r32) in enumerate([(depth, dr, dr32), (centers, cr, cr32)] + list(zip(attn, ar, ar32))):
        _check_fwd_conditioned(f"output {i}", a, r, r32)
    dy = torch.from_numpy(rng_array(tuple(dr.shape), 85))
    (depth * dy.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()

    def loss_fn(P):
        d, _, _ = odf.depthformer_v8_full(P, img.to(P["decoder.aux_embedding"].dtype), opt, 1e-3, 10.0)
        (d * dy.to(d.dtype)).sum().backward()

    assert _check_param_grads(m, sd, loss_fn, rel=1e-3) > 0


def _fwd(sd, dtype, fn):
    with torch.no_grad():
        return fn({k: v.to(dtype) if torch.is_floating_point(v) else v for k, v in sd.items()}, dtype)
