"""Which module's forward output first differs between the fused-dropout bf16 Depthformer
step and the unfused one (MDEMI_FUSE_DROPOUT) -- a bisection aid for
tests/test_dropout_fused_gpu.py.   python tools/diag_fuse.py [fp32|bf16]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402

from mdemi import functional as mf  # noqa: E402
from mdemi.model.Depthformer import DepthformerV8  # noqa: E402
from oracle.weights import closed_form_fill, rng_array  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
DEV = "cuda"
opt = {"hidden_dim": 64, "num_heads": 4, "num_bins": 64, "num_aux": 32, "img_size": [128, 160],
       "attn_drop_prob": 0.1, "drop_prob": 0.2}
torch.manual_seed(0)
m = DepthformerV8.build(opt, 1e-3, 10.0)
sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
closed_form_fill(sd, seed=0.37, scale=0.03)
img = torch.from_numpy(rng_array((2, 3, 128, 160), 41)).float().to(DEV)
m = m.to(DEV).train()
rec = {}
calls = []


def hook(name):
    def f(mod, inp, out):
        outs = out if isinstance(out, (tuple, list)) else (out,)
        rec.setdefault(name, []).append([o.detach().clone() for o in outs if torch.is_tensor(o)])
    return f


for n, mod in m.named_modules():
    if n:
        mod.register_forward_hook(hook(n))
orig_att = mf.attention


def att(*a, **k):
    o, p = orig_att(*a, **k)
    calls.append((o.detach().clone(), p.detach().clone()))
    return o, p


mf.attention = att
import mdemi.model.Depthformer.luna_layer as ll  # noqa: E402
import mdemi.model.Depthformer.self_attention as sa  # noqa: E402
ll.mf.attention = att
sa.mf.attention = att


def run(fuse):
    rec.clear()
    calls.clear()
    mf._FUSE_DROP[0] = fuse
    m.load_state_dict({k: v.to(DEV) for k, v in sd.items()})
    mf._drop_counter[0] = 0
    torch.manual_seed(123)
    with torch.no_grad(), mf.matmul_precision(prec):
        m(img)
    torch.cuda.synchronize()
    return dict(rec), list(calls)


r0, c0 = run(False)
r1, c1 = run(True)
for i, ((o0, p0), (o1, p1)) in enumerate(zip(c0, c1)):
    print(f"attention call {i}: P equal {torch.equal(p0, p1)}, out equal {torch.equal(o0, o1)} "
          f"max|dout| {(o0 - o1).abs().max().item():.3e}")
for n in r0:
    for k, (a, b) in enumerate(zip(r0[n], r1[n])):
        bad = [j for j, (x, y) in enumerate(zip(a, b)) if not torch.equal(x, y)]
        if bad:
            print("first differing module output:", n, "call", k, "outputs", bad,
                  [(a[j] - b[j]).abs().max().item() for j in bad])
            sys.exit(0)
print("all module outputs equal")
