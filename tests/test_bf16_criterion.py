"""The bf16 gradient acceptance rule (tests/bf16_criterion.py) is falsifiable (CPU).

On the well-conditioned Depthformer v8 case the at-size GPU test uses (oracle.weights.
fanin_fill, BatchNorm on running statistics), but small (hidden 64, 128x160): a second
independent rounding draw -- the fp32 bf16-emulating oracle run on an input perturbed by
2^-22 relative, which moves operands across bf16 rounding boundaries just as the GPU's own
fp32 summation orders do -- passes the rule for every gradient, and the same draw with one
Luna projection's weight gradient scaled by 1.05 (or one bias gradient dropped to zero)
fails it.  References: model/Depthformer/decoder_v8.py:97-171, luna_layer.py:181-259."""
import contextlib

import pytest
import torch

import bf16_criterion as C

OPT = {"hidden_dim": 64, "num_heads": 4, "num_bins": 64, "num_aux": 32, "img_size": [128, 160],
       "attn_drop_prob": 0.0, "drop_prob": 0.0}


@pytest.fixture(scope="module")
def grads():
    return compute_grads()


def compute_grads():
    from oracle import bf16emu, bnmode
    from oracle import depthformer as odf
    from oracle.weights import fanin_fill, rng_array
    from mdemi.model.Depthformer import DepthformerV8
    torch.set_num_threads(8)
    with torch.device("meta"):
        m = DepthformerV8.build(OPT, 1e-3, 10.0)
    sd = {k: torch.empty(v.shape, dtype=v.dtype) for k, v in m.state_dict().items()}
    fanin_fill(sd, gains=C.conditioned_gains())
    img = torch.from_numpy(rng_array((2, 3, 128, 160), 84)).double()
    dy = torch.from_numpy(rng_array((2, 1, 64, 80), 85)).double()

    def run(dtype, emulate, perturb=False):
        P = {k: (v.to(dtype).clone().requires_grad_(True) if torch.is_floating_point(v) else v)
             for k, v in sd.items()}
        x = img
        if perturb:
            x = x * (1 + 2.0 ** -22 * torch.from_numpy(rng_array(tuple(x.shape), 99)).double())
        with (bf16emu.enabled() if emulate else contextlib.nullcontext()), bnmode.eval_bn():
            d, c, a = odf.depthformer_v8_full(P, x.to(dtype), OPT, 1e-3, 10.0)
            assert d.shape == dy.shape
            (d * dy.to(dtype)).sum().backward()
        outs = [t.detach().double() for t in [d, c] + list(a)]
        return {k: p.grad.detach().double() for k, p in P.items() if torch.is_tensor(p) and p.grad is not None}, outs

    res = {"o64": run(torch.float64, True), "o32": run(torch.float32, True),
           "draw": run(torch.float32, True, perturb=True), "plain": run(torch.float64, False)}
    out = {k: v[0] for k, v in res.items()}
    out["outputs"] = {k: v[1] for k, v in res.items()}
    return out


OUT_NAMES = ["depth", "centers"] + [f"attn{k}" for k in range(8)]


def test_independent_draw_passes(grads):
    r = C.judge(grads["draw"], grads["o64"], grads["o32"], grads["plain"])
    print(f"worst: {r['rows'][:3]}; {len(r['noisy'])} of {r['checked']} noise-dominated")
    assert not r["bad"], r["bad"]
    assert r["checked"] == len(grads["o64"]) > 600
    assert len(r["noisy"]) < C.MAX_NOISY_FRACTION * r["checked"]


@pytest.mark.parametrize("proj", ["v1_proj", "o1_proj", "v2_proj", "o2_proj"])
def test_scaled_luna_gradient_fails(grads, proj):
    """At this small size the rule holds the Luna layer-0 projections to 3.6-4.2 % (the draw
    sits 0.7-0.8 % from o64), so a 5 % error fails it; at the benchmark size (480x640,
    test_bf16_graph_gpu) every Luna value/output projection is held to 1.7-2.9 %."""
    k = f"decoder.luna_layers.0.luna_attn.{proj}.weight"
    wrong = dict(grads["draw"])
    wrong[k] = wrong[k] * 1.05
    r = C.judge(wrong, grads["o64"], grads["o32"], grads["plain"])
    assert [b[0] for b in r["bad"]] == [k], r["bad"]


def test_independent_draw_outputs_pass(grads):
    o = grads["outputs"]
    assert len(o["draw"]) == len(OUT_NAMES)
    r = C.judge_outputs(OUT_NAMES, o["draw"], o["o64"], o["o32"])
    print(f"outputs, worst: {r['rows'][:3]}")
    assert not r["bad"], r["bad"]


@pytest.mark.parametrize("which", ["depth", "centers"])
def test_output_off_by_two_percent_fails(grads, which):
    """The depth map or the bin centres scaled by 1.02 fail the output rule (their draws sit
    0.04-0.16 % from o64 here)."""
    o = grads["outputs"]
    i = OUT_NAMES.index(which)
    wrong = list(o["draw"])
    wrong[i] = wrong[i] * 1.02
    r = C.judge_outputs(OUT_NAMES, wrong, o["o64"], o["o32"])
    assert [b[0] for b in r["bad"]] == [which], r["bad"]


def test_attention_maps_are_noise_dominated_draws(grads):
    """Why attention maps get the conditioned check: here the two emulations' maps differ by
    more than 2 % (so rule (1) passes a map scaled by 1.02), as much as bf16 moves them from
    the un-rounded model."""
    o = grads["outputs"]
    for k in range(8):
        i = OUT_NAMES.index(f"attn{k}")
        assert C._l2(o["o32"][i] - o["o64"][i]) > 5e-3 * C._l2(o["o64"][i])
    wrong = list(o["draw"])
    wrong[2] = wrong[2] * 1.02
    assert not C.judge_outputs(OUT_NAMES, wrong, o["o64"], o["o32"])["bad"]


def _attn_case(seed=3, scale=0.25):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(2, 4, 96, 64, generator=g) * 2.0
    k = torch.randn(2, 4, 80, 64, generator=g) * 2.0
    ref = C.attention_reference(q, k, scale)
    # what the GPU computes: fp32 logits of the exact bf16 products, fp32 softmax
    q16, k16 = q.to(torch.bfloat16).float(), k.to(torch.bfloat16).float()
    p32 = torch.softmax(scale * q16 @ k16.transpose(-1, -2), dim=-1)
    return p32, ref


def test_attention_given_inputs_passes():
    p32, ref = _attn_case()
    ok, rel, rows = C.judge_attention(p32, ref)
    assert ok, (rel, rows)
    assert rel < 1e-5


@pytest.mark.parametrize("kind", ["scaled", "mixed", "unrounded_operands"])
def test_attention_off_by_two_percent_fails(kind):
    """A map scaled by 1.02, one with 2 % of each row moved to other keys (rows still sum to
    one), and one computed from the un-rounded fp32 q / k (a kernel that skipped the bf16
    rounding) all fail the conditioned attention check."""
    p32, ref = _attn_case()
    if kind == "scaled":
        bad = p32 * 1.02
    elif kind == "mixed":
        bad = 0.98 * p32 + 0.02 * torch.roll(p32, 7, dims=-1)
    else:
        g = torch.Generator().manual_seed(3)
        q = torch.randn(2, 4, 96, 64, generator=g) * 2.0
        k = torch.randn(2, 4, 80, 64, generator=g) * 2.0
        bad = torch.softmax(0.25 * q @ k.transpose(-1, -2), dim=-1)
    ok, rel, rows = C.judge_attention(bad, ref)
    assert not ok, (kind, rel, rows)


def test_missing_bias_term_fails(grads):
    k = "decoder.luna_layers.3.feed_forward.fc2.bias"
    wrong = dict(grads["draw"])
    wrong[k] = torch.zeros_like(wrong[k])
    r = C.judge(wrong, grads["o64"], grads["o32"], grads["plain"])
    assert [b[0] for b in r["bad"]] == [k], r["bad"]


def test_shift_invariant_bias_held_in_size(grads):
    """A key-projection bias gradient (exactly zero) may be rounding residue, not more."""
    k = "decoder.luna_layers.3.luna_attn.k1_proj.bias"
    assert C.SHIFT_INVARIANT.search(k)
    wrong = dict(grads["draw"])
    wrong[k] = torch.full_like(wrong[k], 1e-2 * grads["o64"][k[:-4] + "weight"].abs().max().item())
    r = C.judge(wrong, grads["o64"], grads["o32"], grads["plain"])
    assert [b[0] for b in r["bad"]] == [k], r["bad"]
