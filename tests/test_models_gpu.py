"""Model-level parity on the GPU: the mdemi modules (libmdemi kernels, NHWC
inside) against golden vectors produced by the reference itself, with the
reference's weights rebuilt from the closed-form fill and identical inputs.
Forward outputs and every parameter/input gradient are compared
(fp32 kernels vs the fp32 reference: tolerances stated per check)."""
import pytest
import torch

from golden_util import Golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
RT_OUT, RT_GRAD = 1e-4, 1e-3


def nchw_to_nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nhwc_to_nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def load_golden_weights(model, g):
    from oracle.weights import closed_form_fill, rng_fill
    sd = model.state_dict()
    cpu = {k: v.detach().cpu().clone() for k, v in sd.items()}
    if g.fill_mode == "rng":
        rng_fill(cpu, seed=int(g.fill[0]), scale=g.fill[1])
    else:
        closed_form_fill(cpu, seed=g.fill[0], scale=g.fill[1])
    for mod in model.modules():  # the fixtures were generated with dropout off (make_golden.prep)
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        if isinstance(mod, torch.nn.MultiheadAttention):
            mod.dropout = 0.0
    with torch.no_grad():
        for k, v in sd.items():
            if torch.is_floating_point(v):
                v.copy_(cpu[k])
    return model


def run_case(g, model, fwd, out_names, out_layouts, in_layouts, no_input_grad=(), vanishing=None):
    """in_layouts/out_layouts: name -> 'nchw' (converted to/from NHWC) or 'same'.
    no_input_grad: inputs the product never differentiates (the input image).
    vanishing: regex of parameters whose exact gradient is zero (fp32 round-off only):
    compared in size (<= 10x the reference's norm), not value."""
    model = load_golden_weights(model.to(DEV), g)
    model.train()
    model.zero_grad(set_to_none=True)
    ins = {}
    for n in g.input_names():
        t = g.input(n, torch.float32)
        if in_layouts.get(n) == "nchw":
            t = nchw_to_nhwc(t)
        ins[n] = t.to(DEV).requires_grad_(True)
    outs = fwd(model, ins)
    if not isinstance(outs, (tuple, list)):
        outs = (outs,)
    loss = 0
    for name, o in zip(out_names, outs):
        oc = nhwc_to_nchw(o) if out_layouts.get(name) == "nchw" else o
        g.check(f"out/{name}", oc.float().cpu(), RT_OUT, 1e-5)
        dy = g.dy(name, oc.shape, torch.float32).to(DEV)
        if out_layouts.get(name) == "nchw":
            dy = nchw_to_nhwc(dy)
        loss = loss + (o * dy).sum()
    loss.backward()
    for n, t in ins.items():
        if n in no_input_grad:
            assert t.grad is None
            continue
        if g.has(f"grad/{n}"):
            gr = nhwc_to_nchw(t.grad) if in_layouts.get(n) == "nchw" else t.grad
            g.check(f"grad/{n}", gr.cpu(), RT_GRAD, 1e-5)
    n_checked = 0
    for k, p in model.named_parameters():
        if vanishing is not None and vanishing.search(k) and (g.has(f"grad/{k}") or f"gsum/{k}" in g.d):
            import numpy as np
            ref = float(np.sqrt(g.d[f"gsum/{k}"][1])) if f"gsum/{k}" in g.d else \
                float(np.linalg.norm(g.d.get(f"grad/{k}", g.d.get(f"sub/grad/{k}"))))
            assert p.grad.double().norm().item() <= 10 * ref + 1e-8, k
            n_checked += 1
        elif g.has(f"grad/{k}"):
            g.check(f"grad/{k}", p.grad.cpu(), RT_GRAD, 1e-5)
            n_checked += 1
        elif f"gsum/{k}" in g.d:
            s = g.d[f"gsum/{k}"]
            gv = p.grad.double().cpu()
            tol = 2e-3
            assert abs(gv.sum().item() - s[0]) <= tol * (s[1] * gv.numel()) ** 0.5 + 1e-6, k
            assert abs((gv * gv).sum().item() - s[1]) <= 2 * tol * s[1] + 1e-12, k
            n_checked += 1
    return n_checked


@pytest.mark.parametrize("hw", [(10, 12), (9, 13)])
def test_swin_basic_layer(hw):
    from mdemi.model.NewCRFs.swin_transformer import BasicLayer, PatchMerging
    H, W = hw
    g = Golden(f"swin_basic_layer_{H}x{W}")
    m = BasicLayer(dim=64, depth=2, num_heads=2, window_size=7, downsample=PatchMerging)

    def fwd(m, i):
        r = m(i["x"], H, W)
        return r[0], r[3]

    assert run_case(g, m, fwd, ["x_out", "x_down"], {}, {}) == len(list(m.parameters()))


def test_swin_window_attention_unshifted_windows():
    """WindowAttention on pre-partitioned windows == 7x7 images, shift 0."""
    from mdemi import functional as mf
    from mdemi.model.NewCRFs.swin_transformer import WindowAttention
    g = Golden("swin_window_attention")
    m = WindowAttention(64, (7, 7), 2)

    def fwd(m, i):
        x = i["x"].reshape(-1, 64)
        a = m.attend(x, 6, 7, 7, 0)
        return mf.linear(a, m.proj.weight, m.proj.bias).view(6, 49, 64)

    run_case(g, m, fwd, ["y"], {}, {})


def test_swin_backbone():
    from mdemi.model.NewCRFs.swin_transformer import SwinTransformer
    g = Golden("swin_backbone")
    m = SwinTransformer(embed_dim=64, depths=[2, 2, 2, 2], num_heads=[2, 4, 8, 16], window_size=7, drop_path_rate=0.0)
    n = run_case(g, m, lambda m, i: m(i["img"]), ["o0", "o1", "o2", "o3"], {f"o{k}": "nchw" for k in range(4)}, {},
                 no_input_grad=("img",))
    assert n == len(list(m.parameters()))


def test_newcrf_layer():
    from mdemi.model.NewCRFs.newcrf_layers import NewCRF
    g = Golden("newcrf_layer")
    m = NewCRF(input_dim=96, embed_dim=128, window_size=7, v_dim=64, num_heads=4)
    run_case(g, m, lambda m, i: m(i["x"], i["v"]), ["y"], {"y": "nchw"}, {"x": "nchw", "v": "nchw"})


def test_psp_head():
    from mdemi.model.NewCRFs.uper_crf_head import PSP
    g = Golden("psp_head")
    m = PSP(in_channels=[16, 32, 64, 128], in_index=[0, 1, 2, 3], pool_scales=(1, 2, 3, 6), channels=512,
            dropout_ratio=0.0, num_classes=32, norm_cfg=dict(type="BN", requires_grad=True), align_corners=False)
    run_case(g, m, lambda m, i: m([i["f0"], i["f1"], i["f2"], i["f3"]]), ["y"], {"y": "nchw"},
             {f"f{k}": "nchw" for k in range(4)})


def test_disp_head():
    from mdemi.model.NewCRFs.NewCRFDepth import DispHead
    g = Golden("disp_head")
    m = DispHead(input_dim=128)
    run_case(g, m, lambda m, i: m(i["x"], 4), ["y"], {"y": "nchw"}, {"x": "nchw"})


def test_newcrfs_tiny07_end_to_end():
    from mdemi.model.NewCRFs import NewCRFDepth
    g = Golden("newcrfs_tiny07")
    m = NewCRFDepth(version="tiny07", max_depth=10.0, drop_path_rate=0.0)
    n = run_case(g, m, lambda m, i: m(i["img"]), ["depth"], {}, {}, no_input_grad=("img",))
    assert n == len(list(m.parameters()))


# ---------------------------------------------------------------------------
# AdaBins (model/Adabins) — EfficientNet-B5 features stand in as stored maps
# ---------------------------------------------------------------------------
class _Const(torch.nn.Module):
    def __init__(self, holder, idx):
        super().__init__()
        self.__dict__["_holder"] = holder
        self.idx = idx

    def forward(self, x):
        return self._holder.get(self.idx, x)


def fake_backend(holder):
    """Module tree walked like gen-efficientnet's; feature k returns holder[k] (NHWC)."""
    m = torch.nn.Module()
    m.conv_stem, m.bn1, m.act1 = _Const(holder, 1), _Const(holder, 2), _Const(holder, 3)
    m.blocks = torch.nn.Sequential(*[_Const(holder, 4 + i) for i in range(7)])
    m.conv_head, m.act2 = _Const(holder, 11), _Const(holder, 12)
    return m


def oracle_grads(g, oracle_fn, out_names, dtype):
    """Oracle forward+backward of L = sum(out * dy) on the golden weights/inputs in `dtype`."""
    P = g.params(dtype)
    for v in P.values():
        if torch.is_floating_point(v):
            v.requires_grad_(True)
    ins = {n: g.input(n, dtype).requires_grad_(True) for n in g.input_names()}
    outs = oracle_fn(P, ins)
    loss = 0
    for name, o in zip(out_names, outs):
        loss = loss + (o * g.dy(name, o.shape, dtype)).sum()
    loss.backward()
    return P, ins


def check_grads_conditioned(g, model, ins, in_layouts, oracle_fn, out_names, slack=20.0):
    """Gradients of deep BatchNorm decoders at batch 1 are ill-conditioned: the reference's own fp32
    gradients differ from fp64 by up to ~3e-2 relative (the pre-BN conv biases, exactly zero in exact
    arithmetic, are pure rounding noise).  So the GPU gradients are held to the fp64 oracle (pinned to
    the reference by tests/test_oracle_golden.py) within `slack` x the fp32 CPU error of the same
    computation, plus 1e-4 relative."""
    P64, I64 = oracle_grads(g, oracle_fn, out_names, torch.float64)
    P32, I32 = oracle_grads(g, oracle_fn, out_names, torch.float32)
    checked = 0
    pairs = [(k, p.grad, P64[k].grad, P32[k].grad) for k, p in model.named_parameters()]
    pairs += [(n, nhwc_to_nchw(t.grad) if in_layouts.get(n) == "nchw" else t.grad, I64[n].grad, I32[n].grad)
              for n, t in ins.items()]
    for k, got, r64, r32 in pairs:
        e_gpu = (got.double().cpu() - r64).abs().max().item()
        e_cpu = (r32.double() - r64).abs().max().item()
        mag = r64.abs().max().item()
        assert e_gpu <= slack * e_cpu + 1e-4 * mag + 1e-9, (k, e_gpu, e_cpu, mag)
        checked += 1
    return checked


def test_adabins_head():
    """UnetAdaptiveBins after the encoder (decoder, mViT, folded conv_out + bin head) vs the reference."""
    from mdemi.model.Adabins import UnetAdaptiveBins
    g = Golden("adabins_head")
    holder = {}
    m = UnetAdaptiveBins(fake_backend(holder), n_bins=256, min_val=1e-3, max_val=10.0)

    def fwd(m, i):
        holder.clear()
        for k, v in i.items():
            holder[int(k[1:])] = v
        return m(torch.zeros(1, 3, 8, 8, device=DEV))

    lay = {k: "nchw" for k in g.input_names()}
    model = load_golden_weights(m.to(DEV), g).train()
    ins = {n: nchw_to_nhwc(g.input(n, torch.float32)).to(DEV).requires_grad_(True) for n in g.input_names()}
    pred, edges = fwd(model, ins)
    g.check("out/pred", pred.float().cpu(), RT_OUT, 1e-5)
    g.check("out/bin_edges", edges.float().cpu(), RT_OUT, 1e-5)
    ((pred * g.dy("pred", pred.shape, torch.float32).to(DEV)).sum() +
     (edges * g.dy("bin_edges", edges.shape, torch.float32).to(DEV)).sum()).backward()
    from oracle import adabins as oab
    n = check_grads_conditioned(g, model, ins, lay, lambda P, i: oab.adabins_head(
        P, {int(k[1:]): v for k, v in i.items()}, 1e-3, 10.0), ["pred", "bin_edges"])
    assert n == len(list(m.parameters())) + len(ins)


def test_mvit():
    from mdemi.model.Adabins import mViT
    g = Golden("mvit")
    m = mViT(128, n_query_channels=128, patch_size=16, dim_out=256, embedding_dim=128, norm="linear")
    n = run_case(g, m, lambda m, i: m(i["x"]), ["bin_widths", "range_maps"], {"range_maps": "nchw"},
                 {"x": "nchw"})
    assert n == len(list(m.parameters()))


def _filled_state(model, seed, scale):
    """Closed-form weights (oracle/weights.py) loaded into `model`; returns the CPU state dict."""
    from oracle.weights import closed_form_fill
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    closed_form_fill(sd, seed=seed, scale=scale)
    model.load_state_dict(sd)
    return sd


def _oracle_run(sd, dtype, loss_fn):
    # fresh leaves every run (a no-op .to() would hand out sd's own tensors, whose .grad then
    # accumulates across runs and turns later casts into non-leaves)
    P = {k: (v.detach().to(dtype).clone().requires_grad_(True) if torch.is_floating_point(v) else v)
         for k, v in sd.items()}
    outs = loss_fn(P)
    return P, outs


def _check_param_grads(model, sd, loss_fn, slack=20.0, rel=1e-4, only=None):
    """GPU parameter gradients vs the fp64 oracle, within `slack` x the fp32 oracle's own error
    (BatchNorm stacks make some gradients -- e.g. biases feeding a BN, exactly zero in exact
    arithmetic -- pure rounding noise) plus `rel` x the gradient's largest magnitude.
    only: check the parameters whose names start with this prefix."""
    P64, _ = _oracle_run(sd, torch.float64, loss_fn)
    P32, _ = _oracle_run(sd, torch.float32, loss_fn)
    n = 0
    for k, p in model.named_parameters():
        if only is not None and not k.startswith(only):
            continue
        r64, r32 = P64[k].grad, P32[k].grad
        if r64 is None:  # no gradient reaches it in the oracle: none (or zero) on the GPU either
            assert p.grad is None or p.grad.abs().max().item() == 0, k
            n += 1
            continue
        e_gpu = (p.grad.double().cpu() - r64).abs().max().item()
        e_cpu = (r32.double() - r64).abs().max().item()
        mag = r64.abs().max().item()
        assert e_gpu <= slack * e_cpu + rel * mag + 1e-9, (k, e_gpu, e_cpu, mag)
        n += 1
    return n


def _no_dropout(model):
    for mod in model.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        if isinstance(mod, torch.nn.MultiheadAttention):
            mod.dropout = 0.0


def _oracle_fwd(sd, dtype, fn):
    with torch.no_grad():
        return fn({k: v.to(dtype) if torch.is_floating_point(v) else v for k, v in sd.items()}, dtype)


def _check_fwd_conditioned(name, got, r64, r32, slack=20.0, rel=1e-4):
    """Forward outputs of the deep BatchNorm encoders (39 MBConv blocks at batch 2 over a few
    pixels per channel, closed-form random weights) are ill-conditioned: the fp32 CPU oracle
    itself strays from fp64 by up to ~1e-3 relative on some outputs.  The GPU output must sit
    within 1e-4 relative of the fp64 oracle, or within `slack` x the fp32 oracle's own error."""
    e_gpu = (got.double().cpu() - r64).abs().max().item()
    e_cpu = (r32.double() - r64).abs().max().item()
    mag = r64.abs().max().item()
    print(f"{name}: gpu err {e_gpu:.3e} = {e_gpu / max(rel * mag, slack * e_cpu):.3f} of the bound (cpu fp32 err {e_cpu:.3e})")
    assert e_gpu <= max(rel * mag, slack * e_cpu) + 1e-9, (name, e_gpu, e_cpu, mag)


def test_efficientnet_b5_encoder_vs_oracle():
    """Restated tf_efficientnet_b5_ap (parity unpinned: third-party, not offline) -- libmdemi vs the
    CPU oracle restatement on the same closed-form weights: features [4,5,6,8,11] and all grads."""
    from mdemi.model.gen_efficientnet import tf_efficientnet_b5_ap, walk_features
    from oracle import efficientnet as oeff
    from oracle.weights import rng_array
    net = tf_efficientnet_b5_ap()
    del net.bn2, net.global_pool, net.classifier
    sd = _filled_state(net, 0.31, 0.05)
    net = net.to(DEV).train()
    img = torch.from_numpy(rng_array((2, 3, 64, 96), 77))
    fg = walk_features(net, img.float().to(DEV), 11)
    dys = {}
    loss_g = 0
    fr, fr32 = (_oracle_fwd(sd, dt, lambda P, dt: oeff.features(P, "", img.to(dt), 11))
                for dt in (torch.float64, torch.float32))
    for k in (4, 5, 6, 8, 11):
        a, r = fg[k], fr[k]
        _check_fwd_conditioned(f"feature {k}", nhwc_to_nchw(a), r, fr32[k])
        dys[k] = torch.from_numpy(rng_array(tuple(r.shape), 100 + k))
        loss_g = loss_g + (nhwc_to_nchw(a) * dys[k].float().to(DEV)).sum()
    loss_g.backward()

    def loss_fn(P):
        f = oeff.features(P, "", img.to(P["conv_stem.weight"].dtype), 11)
        loss = sum((f[k] * dys[k].to(f[k].dtype)).sum() for k in dys)
        loss.backward()

    # 1e-3: tools/diag_effnet.py on the box measured the GPU/fp32-CPU error ratio over all 506
    # encoder gradients at median 3.2, worst 49 (a SqueezeExcite reduce bias: 6.9e-4 relative);
    # the CPU's BatchNorm/reductions accumulate in fp64, the GPU's partial sums in fp32.
    assert _check_param_grads(net, sd, loss_fn, rel=1e-3) == len(list(net.parameters()))


def test_adabins_end_to_end_vs_oracle():
    """Whole UnetAdaptiveBins (restated B5 encoder + reference-pinned head) vs the CPU oracle."""
    from mdemi.model.Adabins import UnetAdaptiveBins
    from oracle import adabins as oab
    from oracle.weights import rng_array
    m = UnetAdaptiveBins.build(256, 1e-3, 10.0)
    sd = _filled_state(m, 0.41, 0.03)
    _no_dropout(m)  # the oracle is deterministic: mViT's transformer dropout (p=0.1) off
    m = m.to(DEV).train()
    img = torch.from_numpy(rng_array((2, 3, 352, 384), 78))
    pred, edges = m(img.float().to(DEV))
    (pr, er), (pr32, er32) = (_oracle_fwd(sd, dt, lambda P, dt: oab.unet_adaptive_bins(P, img.to(dt), 1e-3, 10.0))
                              for dt in (torch.float64, torch.float32))
    _check_fwd_conditioned("pred", pred, pr, pr32)
    _check_fwd_conditioned("bin_edges", edges, er, er32)
    dy = torch.from_numpy(rng_array(tuple(pr.shape), 79))
    (pred * dy.float().to(DEV)).sum().backward()

    def loss_fn(P):
        p, _ = oab.unet_adaptive_bins(P, img.to(P["conv_out.0.weight"].dtype), 1e-3, 10.0)
        (p * dy.to(p.dtype)).sum().backward()

    # gradients through the restated B5 encoder: same 1e-3 basis as test_efficientnet_b5_encoder_vs_oracle
    assert _check_param_grads(m, sd, loss_fn, rel=1e-3) == len(list(m.parameters()))


# ---------------------------------------------------------------------------
# Depthformer v8 (model/Depthformer)
# ---------------------------------------------------------------------------
DFV8_OPT = {"hidden_dim": 64, "num_heads": 4, "num_bins": 32, "num_aux": 16, "img_size": [64, 96],
            "attn_drop_prob": 0.0, "drop_prob": 0.0}


def test_depthformer_v8_decoder_and_head():
    """Decoder (Luna x4, ViT aux layer, ResConvBN with replicate padding, shoot heads) + bin head
    vs the reference, EfficientNet features as stored maps; depth, centres and all 8 attention maps."""
    from mdemi.model.Depthformer import DepthformerV8
    g = Golden("depthformer_v8")
    holder = {}
    m = DepthformerV8(fake_backend(holder), DFV8_OPT, min_depth=1e-3, max_depth=10.0)

    def fwd(m, i):
        holder.clear()
        for k, v in i.items():
            holder[int(k[1:])] = v
        depth, centers, attn = m(torch.zeros(2, 3, 8, 8, device=DEV))
        return (depth, centers) + tuple(attn)

    n = run_case(g, m, fwd, ["depth", "centers"] + [f"attn{k}" for k in range(8)], {},
                 {k: "nchw" for k in g.input_names()})
    assert n == len(list(m.parameters()))


def test_depthformer_v8_end_to_end_vs_oracle():
    """Whole DepthformerV8 (restated B5 encoder + reference-pinned decoder) vs the CPU oracle."""
    from mdemi.model.Depthformer import DepthformerV8
    from oracle import depthformer as odf
    from oracle.weights import rng_array
    opt = {"hidden_dim": 64, "num_heads": 4, "num_bins": 64, "num_aux": 32, "img_size": [128, 160],
           "attn_drop_prob": 0.0, "drop_prob": 0.0}
    m = DepthformerV8.build(opt, 1e-3, 10.0)
    sd = _filled_state(m, 0.51, 0.03)
    m = m.to(DEV).train()
    img = torch.from_numpy(rng_array((2, 3, 128, 160), 80))
    depth, centers, attn = m(img.float().to(DEV))
    (dr, cr, ar), (dr32, cr32, ar32) = (
        _oracle_fwd(sd, dt, lambda P, dt: odf.depthformer_v8_full(P, img.to(dt), opt, 1e-3, 10.0))
        for dt in (torch.float64, torch.float32))
    for i, (a, r, r32) in enumerate([(depth, dr, dr32), (centers, cr, cr32)] + list(zip(attn, ar, ar32))):
        _check_fwd_conditioned(f"output {i}", a, r, r32)
    dy = torch.from_numpy(rng_array(tuple(dr.shape), 81))
    (depth * dy.float().to(DEV)).sum().backward()

    def loss_fn(P):
        d, _, _ = odf.depthformer_v8_full(P, img.to(P["decoder.aux_embedding"].dtype), opt, 1e-3, 10.0)
        (d * dy.to(d.dtype)).sum().backward()

    # gradients through the restated B5 encoder: same 1e-3 basis as test_efficientnet_b5_encoder_vs_oracle
    assert _check_param_grads(m, sd, loss_fn, rel=1e-3) == len(list(m.parameters()))


def test_flip_eval_metrics_newcrfs_tiny07():
    """GPU evaluation path (mdemi.evaluate): model -> flip-eval -> 9 metrics -> running mean,
    against the fp64 oracle forward on the image and its mirror, averaged, and the reference's
    metric formulas (oracle.metrics.compute_errors) over the NYU eigen crop."""
    import numpy as np

    from mdemi.evaluate import evaluate
    from mdemi.model.NewCRFs import NewCRFDepth
    from oracle import metrics as omet
    from oracle import newcrfs as onc
    from oracle.weights import closed_form_fill, rng_array

    m = NewCRFDepth(version="tiny07", max_depth=10.0, drop_path_rate=0.0)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    closed_form_fill(sd, seed=0.3, scale=0.02)
    m.load_state_dict(sd)
    m = m.to(DEV)
    H, W = 96, 128
    img = torch.from_numpy(rng_array((2, 3, H, W), 21))
    g = torch.Generator().manual_seed(5)
    gt = torch.rand(2, 1, H, W, generator=g, dtype=torch.float64) * 9.0 + 0.5
    gt[:, :, :10] = 0.0  # invalid rows
    sd64 = {k: v.double() if torch.is_floating_point(v) else v for k, v in sd.items()}
    # evaluate() runs model.eval(): BatchNorm on running statistics in the oracle too
    ref = onc.newcrf_depth(sd64, img.double(), "tiny07", max_depth=10.0, bn_eval=True)
    ref_f = onc.newcrf_depth(sd64, torch.flip(img.double(), dims=[-1]), "tiny07", max_depth=10.0, bn_eval=True)
    ref = 0.5 * (ref + torch.flip(ref_f, dims=[-1]))
    eval_opt = {"min_depth_eval": 1e-3, "max_depth_eval": 10.0, "garg_crop": False, "eigen_crop": True,
                "flip_eval": True}
    # NYU eigen crop at 96x128 is the full-frame rectangle (45:471, 41:601) -- use KITTI's relative one
    got = evaluate(m, [(img.float().to(DEV), gt.float().to(DEV))], eval_opt, "KITTI")
    mask = omet.cal_eval_mask(eval_opt, gt[0, 0].numpy(), "KITTI")
    want = {}
    for i in range(2):
        p = np.clip(ref[i, 0].numpy(), 1e-3, 10.0)
        gi = gt[i, 0].numpy()
        valid = mask & (gi > 1e-3) & (gi < 10.0)
        e = omet.compute_errors(gi[valid], p[valid])
        for k, v in e.items():
            want[k] = want.get(k, 0.0) + float(v) / 2
    for k in ("a1", "a2", "a3", "abs_rel", "sq_rel", "rmse", "rmse_log", "silog", "log_10"):
        # depth within 1e-4 rel (north_star); metrics follow; threshold metrics may flip one pixel
        tol = 2.0 / mask.sum() if k in ("a1", "a2", "a3") else 1e-4 * abs(want[k]) + 1e-7
        assert abs(got[k] - want[k]) <= tol, (k, got[k], want[k])


@pytest.mark.parametrize("H,W,max_depth,data_type", [(480, 640, 10.0, "NYU"), (352, 1216, 80.0, "KITTI")])
def test_large07_full_size_depth_and_abs_rel_parity(H, W, max_depth, data_type):
    """north_star's parity bar at the benchmark configurations: NeW-CRFs Swin-L (large07) forward
    on one full NYU 480x640 / KITTI 352x1216 crop through libmdemi vs the fp64 oracle restatement
    (pinned to the reference by the golden fixtures): depth within 1e-4 relative, and abs_rel /
    RMSE over the eigen crop equal to 4 significant figures."""
    import numpy as np

    from mdemi.model.NewCRFs import NewCRFDepth
    from mdemi.utils.depth_utils import tcompute_errors_gpu
    from oracle import metrics as omet
    from oracle import newcrfs as onc
    from oracle.weights import closed_form_fill, rng_array

    torch.set_num_threads(16)
    m = NewCRFDepth(version="large07", max_depth=max_depth, drop_path_rate=0.0)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    closed_form_fill(sd, seed=0.11, scale=0.02)
    m.load_state_dict(sd)
    m = m.to(DEV).train()  # training-mode BatchNorm, as the oracle
    img = torch.from_numpy(rng_array((1, 3, H, W), 31))
    with torch.no_grad():
        depth = m(img.float().to(DEV)).double().cpu()
        ref = onc.newcrf_depth({k: v.double() if torch.is_floating_point(v) else v for k, v in sd.items()},
                               img.double(), "large07", max_depth=max_depth)
    err = (depth - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-4 * scale, f"depth max|err| {err:.3e} vs max {scale:.3e}"
    g = torch.Generator().manual_seed(9)
    gt = ref * (0.8 + 0.4 * torch.rand(ref.shape, generator=g, dtype=torch.float64))
    eo = {"min_depth_eval": 1e-3, "max_depth_eval": max_depth, "garg_crop": False, "eigen_crop": True}
    got = tcompute_errors_gpu(depth.float().to(DEV), gt.float().to(DEV), eo, data_type)[0]
    mask = omet.cal_eval_mask(eo, gt[0, 0].numpy(), data_type)
    gi, pi = gt[0, 0].numpy(), np.clip(ref[0, 0].numpy(), 1e-3, max_depth)
    valid = mask & (gi > 1e-3) & (gi < max_depth)
    want = omet.compute_errors(gi[valid], pi[valid])
    for k in ("abs_rel", "rmse"):
        assert float(f"{got[k]:.4g}") == float(f"{want[k]:.4g}"), (k, got[k], want[k])


def test_graphed_predictor_matches_eager():
    """hipGraph-captured inference (flip-eval) replays bit-identically to the eager path, for two
    different inputs through the same capture."""
    from mdemi.evaluate import GraphedPredictor, predict_depth
    from mdemi.model.NewCRFs import NewCRFDepth
    from oracle.weights import closed_form_fill, rng_array

    m = NewCRFDepth(version="tiny07", max_depth=10.0, drop_path_rate=0.0)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    closed_form_fill(sd, seed=0.5, scale=0.02)
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    a = torch.from_numpy(rng_array((2, 3, 64, 96), 3)).float().to(DEV)
    b = torch.from_numpy(rng_array((2, 3, 64, 96), 4)).float().to(DEV)
    gp = GraphedPredictor(m, a, flip_eval=True)
    for x in (a, b, a):
        got = gp(x)
        want = predict_depth(m, x, flip_eval=True)
        torch.cuda.synchronize()
        assert torch.equal(got, want)
    # eager work at a larger shape after the capture grows the shared workspaces (split-K
    # slabs, attention scratch): the graph must keep replaying into buffers that stay alive
    big = torch.from_numpy(rng_array((4, 3, 128, 192), 5)).float().to(DEV)
    m.train()
    (m(big) * 1.0).sum().backward()
    m.eval()
    m.zero_grad(set_to_none=True)
    want_big = predict_depth(m, big, flip_eval=True)
    junk = [torch.full((1 << 20,), float("nan"), device=DEV) for _ in range(8)]  # reuse freed blocks
    for x in (a, b):
        got = gp(x)
        want = predict_depth(m, x, flip_eval=True)
        torch.cuda.synchronize()
        assert torch.equal(got, want)
    assert torch.isfinite(want_big).all() and len(junk) == 8
