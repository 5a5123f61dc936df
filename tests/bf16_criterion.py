"""Acceptance rule for a bf16 (BASELINE configs[4]) train step's gradients against the
bf16-emulating oracle (oracle/bf16emu.py) -- test infrastructure, shared by
test_bf16_graph_gpu.py (the GPU at 480x640) and test_bf16_criterion.py (the rule itself on
the CPU, including that it rejects a wrong gradient).

bf16 rounds every GEMM operand to 8 mantissa bits, and rounding is discontinuous: two
computations of the same bf16 model that differ only at fp32 level (a summation order, one
ulp of an input) round some operands differently, so their gradients differ by an amount
set by the model's conditioning, not by their arithmetic.  The oracle measures that amount
directly: o64 is the bf16-operand computation in fp64 (its exact value), o32 the same in
fp32 -- one independent rounding draw.  The GPU is another draw, so per parameter

    ||gpu - o64|| <= DRAW_FACTOR * ||o32 - o64|| + REL_FLOOR * ||o64||          (1)

The bound is a property of the case: on a well-conditioned network (oracle.weights.
fanin_fill, BatchNorm on running statistics) o32 sits ~1 % from o64, so (1) holds the GPU to
a few percent per gradient and a gradient off by 5 % fails it (tests/test_bf16_criterion.py).
On an ill-conditioned one (rank-2 closed-form weights, train-mode BatchNorm over batch 2)
||o32 - o64|| is the size of the gradient itself and (1) says nothing -- `noisy` counts
those (bf16 noise n = ||o64 - plain|| / ||o64|| >= NOISE_DOMINATED, plain = the un-rounded
fp64 model), and the at-size test requires fewer than MAX_NOISY_FRACTION of them.

The forward outputs (depth, bin centres and each attention map) are held to the same rule (1)
(`judge_outputs`), so an output off by 2 % fails too.

Key-projection biases (SHIFT_INVARIANT) have an exact gradient of zero (softmax is
invariant to a shift of every logit of a row); what any computation returns for them is
rounding residue, so they are held in size instead:

    ||plain|| <= 1e-9 ||plain of the same attention's value-projection bias||
                                          (checked: it really is zero)
    ||gpu||   <= DRAW_FACTOR * max(||o64||, ||o32||) + SIBLING_FLOOR ||W|| / sqrt(fan_in)  (2)

with W the sibling weight's o64 gradient: the floor is a hundredth of one input feature's
share of it, a scale that does not depend on the bias gradient's own cancellation.
"""
import re

import torch

DRAW_FACTOR = 3.0
REL_FLOOR = 2e-3
NOISE_DOMINATED = 0.1
MAX_NOISY_FRACTION = 0.10
SIBLING_FLOOR = 1e-2
SHIFT_INVARIANT = re.compile(r"(k1_proj|k2_proj|key_proj)\.bias$")
_VALUE_OF = {"k1_proj": "v1_proj", "k2_proj": "v2_proj", "key_proj": "value_proj"}


def _l2(t):
    return torch.linalg.norm(t.double().reshape(-1)).item()


def judge(gpu, o64, o32, plain):
    """gpu, o64, o32, plain: {parameter name: gradient}.  Returns a dict:
    bad     -- [(name, error, bound)] of gradients outside (1) / (2)
    noisy   -- names whose bf16 noise n >= NOISE_DOMINATED
    rows    -- [(error / bound, name, error, bound, n)] for every gradient, worst first
    checked -- number of gradients judged."""
    bad, noisy, rows = [], [], []
    for k, r64 in o64.items():
        g, r32, p = gpu[k].double(), o32[k].double(), plain[k].double()
        r64 = r64.double()
        n64 = _l2(r64)
        n = _l2(r64 - p) / (n64 + 1e-300)
        if n >= NOISE_DOMINATED:
            noisy.append(k)
        if SHIFT_INVARIANT.search(k):
            sib = k[:-len("bias")] + "weight"
            val = _VALUE_OF[SHIFT_INVARIANT.search(k).group(1)]
            vb = k[:SHIFT_INVARIANT.search(k).start()] + val + ".bias"
            if sib not in o64 or vb not in plain or _l2(p) > 1e-9 * _l2(plain[vb]):
                bad.append((k, _l2(p), "exact gradient expected to vanish"))
                continue
            w = o64[sib].double()
            err, bound = _l2(g), DRAW_FACTOR * max(n64, _l2(r32)) + SIBLING_FLOOR * _l2(w) / w[0].numel() ** 0.5
        else:
            err, bound = _l2(g - r64), DRAW_FACTOR * _l2(r32 - r64) + REL_FLOOR * n64
        rows.append((err / (bound + 1e-300), k, err, bound, n))
        if not err <= bound:
            bad.append((k, err, bound))
    rows.sort(reverse=True)
    return {"bad": bad, "noisy": noisy, "rows": rows, "checked": len(rows)}


def judge_outputs(names, gpu, o64, o32):
    """The same draw rule (1) for the forward outputs (depth, bin centres, attention maps):
    every output, flattened, is one more rounding draw of the bf16 computation.  Returns
    {"bad": [(name, error, bound)], "rows": [(error / bound, name, error, bound)] worst first}."""
    bad, rows = [], []
    for k, g, r64, r32 in zip(names, gpu, o64, o32):
        g, r64, r32 = g.detach().double().cpu(), r64.double(), r32.double()
        err, bound = _l2(g - r64), DRAW_FACTOR * _l2(r32 - r64) + REL_FLOOR * _l2(r64)
        rows.append((err / (bound + 1e-300), k, err, bound))
        if not err <= bound:
            bad.append((k, err, bound))
    rows.sort(reverse=True)
    return {"bad": bad, "rows": rows}


ATTN_REL_L2 = 1e-3   # attention map vs softmax of its own bf16 operands, relative L2
ATTN_ROW_SUM = 1e-5  # |sum of a probability row - 1|


def attention_reference(q, k, scale):
    """P = softmax(scale * bf16(q) bf16(k)^T) in fp64 -- the attention map a bf16 step must
    return GIVEN the q / k it computed ([..., S, d] each; rounded to bf16 here as the QK^T GEMM
    rounds its operands)."""
    q16 = q.detach().cpu().to(torch.bfloat16).double()
    k16 = k.detach().cpu().to(torch.bfloat16).double()
    return torch.softmax(scale * q16 @ k16.transpose(-1, -2), dim=-1)


def judge_attention(p_gpu, p_ref):
    """Attention maps conditioned on their own inputs.  Upstream bf16 rounding moves a Luna
    map by 3-9 % between two equally valid draws (the fp32 and fp64 emulations, at 128x160:
    tests/test_bf16_criterion.py), so the draw rule (1) cannot see a 2 % error in one; given
    the q / k the GPU itself produced, the map is a deterministic fp32 softmax of exact bf16
    products, so it is held to ATTN_REL_L2 relative L2 and every row to sum to 1.  Returns
    (ok, relative L2, worst row-sum error)."""
    g = p_gpu.detach().double().cpu()
    rel = (_l2(g - p_ref) / (_l2(p_ref) + 1e-300))
    rows = (g.sum(-1) - 1.0).abs().max().item()
    return rel <= ATTN_REL_L2 and rows <= ATTN_ROW_SUM, rel, rows


def conditioned_gains():
    """oracle.weights.fanin_fill gains of the well-conditioned configs[4] case: the bin-logit
    conv x32 (peaked, not uniform, bin probabilities: the centre gradients are then not a
    cancellation of near-equal terms) and every attention query/key projection x4 (with
    variance-preserving weights the Luna attentions are uniform to 1e-7, so their query/key
    gradients are a cancellation that bf16 rounds to exactly zero)."""
    g = {"decoder.bin_predictor.2.": 32.0, "decoder.aux_layer.self_attn.query_proj.": 4.0,
         "decoder.aux_layer.self_attn.key_proj.": 4.0}
    for i in range(4):
        for n in ("q1", "k1", "q2", "k2"):
            g[f"decoder.luna_layers.{i}.luna_attn.{n}_proj."] = 4.0
    return g
