"""Diagnostic: per-parameter gradient error of the AdaBins head (golden weights/inputs) for
libmdemi (fp32 GPU) and the CPU oracle in fp32, both against the CPU oracle in fp64."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "monocular-depth-estimation_amd")]
from golden_util import Golden  # noqa: E402
from oracle import adabins as oab  # noqa: E402
import test_models_gpu as T  # noqa: E402

g = Golden("adabins_head")


def oracle(dt):
    P = g.params(dt)
    for v in P.values():
        if torch.is_floating_point(v):
            v.requires_grad_(True)
    ins = {n: g.input(n, dt).requires_grad_(True) for n in g.input_names()}
    pred, edges = oab.adabins_head(P, {int(k[1:]): v for k, v in ins.items()}, 1e-3, 10.0)
    ((pred * g.dy("pred", pred.shape, dt)).sum() + (edges * g.dy("bin_edges", edges.shape, dt)).sum()).backward()
    return P, ins


P64, I64 = oracle(torch.float64)
P32, _ = oracle(torch.float32)
from mdemi.model.Adabins import UnetAdaptiveBins  # noqa: E402
holder = {}
m = UnetAdaptiveBins(T.fake_backend(holder), n_bins=256, min_val=1e-3, max_val=10.0)
m = T.load_golden_weights(m.to("cuda"), g).train()
ins = {n: T.nchw_to_nhwc(g.input(n, torch.float32)).cuda().requires_grad_(True) for n in g.input_names()}
for k, v in ins.items():
    holder[int(k[1:])] = v
pred, edges = m(torch.zeros(1, 3, 8, 8, device="cuda"))
((pred * g.dy("pred", pred.shape, torch.float32).cuda()).sum() +
 (edges * g.dy("bin_edges", edges.shape, torch.float32).cuda()).sum()).backward()
for k, p in m.named_parameters():
    r = P64[k].grad
    mag = r.abs().max().item() + 1e-30
    e_gpu = (p.grad.double().cpu() - r).abs().max().item() / mag
    e_cpu = (P32[k].grad.double() - r).abs().max().item() / mag
    flag = "  <==" if e_gpu > 5 * max(e_cpu, 1e-6) else ""
    print(f"{k:60s} gpu {e_gpu:.2e} cpu32 {e_cpu:.2e}{flag}")
for n in ins:
    r = I64[n].grad
    mag = r.abs().max().item()
    e_gpu = (T.nhwc_to_nchw(ins[n].grad).double().cpu() - r).abs().max().item() / mag
    print(f"input {n}: gpu {e_gpu:.2e}")
