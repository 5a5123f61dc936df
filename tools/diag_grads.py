"""Diagnostic: per-parameter gradient error of a full-size train-step backward against the
fp64 / fp32 CPU oracle (tests/test_fullsize_grads_gpu.py setup), worst ratios first.
    python tools/diag_grads.py adabins|depthformer|large07 [H W]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "monocular-depth-estimation_amd")]
from test_models_gpu import DEV, _filled_state, _no_dropout, _oracle_run  # noqa: E402
from oracle.weights import rng_array  # noqa: E402

torch.set_num_threads(16)
which = sys.argv[1]
H, W = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (480, 640)
if which == "adabins":
    from mdemi.model.Adabins import UnetAdaptiveBins
    from oracle import adabins as oab
    m = UnetAdaptiveBins.build(256, 1e-3, 10.0)
    sd = _filled_state(m, 0.43, 0.03)
    _no_dropout(m)
    img = torch.from_numpy(rng_array((2, 3, H, W), 82))

    def run_oracle(P, x):
        return oab.unet_adaptive_bins(P, x, 1e-3, 10.0)[0]
m = m.to(DEV).train()
pred = m(img.float().to(DEV))[0]
dy = torch.from_numpy(rng_array(tuple(pred.shape), 83))
(pred * dy.float().to(DEV)).sum().backward()
torch.cuda.synchronize()


def loss_fn(P):
    dt = next(v.dtype for v in P.values() if torch.is_floating_point(v))
    (run_oracle(P, img.to(dt)) * dy.to(dt)).sum().backward()


P64, _ = _oracle_run(sd, torch.float64, loss_fn)
P32, _ = _oracle_run(sd, torch.float32, loss_fn)
rows = []
for k, p in m.named_parameters():
    r64, r32 = P64[k].grad, P32[k].grad
    if r64 is None:
        continue
    e_gpu = (p.grad.double().cpu() - r64).abs().max().item()
    e_cpu = (r32.double() - r64).abs().max().item()
    mag = r64.abs().max().item() + 1e-30
    lim = 20 * e_cpu + 1e-3 * mag + 1e-9
    rows.append((e_gpu / lim, k, e_gpu / mag, e_cpu / mag, tuple(p.shape)))
rows.sort(reverse=True)
for r in rows[:40]:
    print(f"{r[0]:8.3f}  gpu_rel {r[2]:.2e}  cpu32_rel {r[3]:.2e}  {r[1]} {r[4]}")
print("failing:", sum(1 for r in rows if r[0] > 1), "of", len(rows))
