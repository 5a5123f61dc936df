"""Deterministic weights and inputs shared by the golden generator and the tests.

closed_form_fill: every floating state_dict entry, in state_dict order, gets
    w[i] = scale * sin(0.7 * i + seed)            (i = running element index)
    1-D ``*weight`` entries (norm scales) and running_var: 1 + scale*sin(...)
so the GPU box can rebuild the exact weights from the formula — and a model
whose state_dict keys/shapes/order differ from the reference's gets different
weights (the fill doubles as a structural check).
"""
import numpy as np
import torch


def closed_form_fill(state_dict, seed=0.0, scale=0.05):
    off = 0
    with torch.no_grad():
        for name, t in state_dict.items():
            if not torch.is_floating_point(t):
                continue
            n = t.numel()
            i = torch.arange(off, off + n, dtype=torch.float64)
            vals = scale * torch.sin(0.7 * i + seed)
            if (t.dim() == 1 and name.endswith("weight")) or name.endswith("running_var"):
                vals = 1.0 + vals
            t.copy_(vals.view_as(t).to(t.dtype))
            off += n
    return off


def rng_fill(state_dict, seed=0, scale=0.05):
    """Well-conditioned alternative to closed_form_fill (full-rank Gaussian weights): entry k
    of the floating state_dict entries, in state_dict order, gets
        w = scale * rng_array(shape, seed * 100003 + k)
    (1 + that for 1-D ``*weight`` entries and running_var).  The closed-form sinusoid makes
    every weight matrix rank 2, which deep BatchNorm/LayerNorm stacks turn into fp32
    round-off amplifiers; tests/golden/make_golden_oda2.py uses this fill."""
    k = 0
    with torch.no_grad():
        for name, t in state_dict.items():
            if not torch.is_floating_point(t):
                continue
            vals = scale * torch.from_numpy(rng_array(tuple(t.shape), int(seed) * 100003 + k)).double()
            if (t.dim() == 1 and name.endswith("weight")) or name.endswith("running_var"):
                vals = 1.0 + vals
            t.copy_(vals.to(t.dtype))
            k += 1
    return k


def fanin_fill(state_dict, seed=7000, gains=None):
    """Variance-preserving Gaussian weights (a well-conditioned network for bf16 parity):
    entry k of the floating state_dict entries, in state_dict order, with r = rng_array(shape,
    seed + k):
        >= 2-D weights          gain / sqrt(fan_in) * r     (fan_in = elements per output row)
        1-D ``*weight`` (norm)  1 + 0.1 * r
        running_var             1 + 0.1 * |r|
        other 1-D (bias, mean)  0.05 * r
    gains: {name prefix: gain} (default 1).  Each layer then passes its input's scale on
    (no activation grows or dies through depth), so bf16 operand rounding stays a
    per-layer 2^-9 perturbation instead of being amplified by rank-deficient weights."""
    k = 0
    gains = gains or {}
    with torch.no_grad():
        for name, t in state_dict.items():
            if not torch.is_floating_point(t):
                continue
            r = torch.from_numpy(rng_array(tuple(t.shape), seed + k)).double()
            if t.dim() >= 2:
                g = next((v for p, v in gains.items() if name.startswith(p)), 1.0)
                vals = g / float(t[0].numel()) ** 0.5 * r
            elif name.endswith("running_var"):
                vals = 1.0 + 0.1 * r.abs()
            elif name.endswith("weight"):
                vals = 1.0 + 0.1 * r
            else:
                vals = 0.05 * r
            t.copy_(vals.to(t.dtype))
            k += 1
    return k


def rng_array(shape, seed=0):
    g = np.random.Generator(np.random.PCG64(seed))
    return g.standard_normal(size=shape).astype(np.float32)
