"""Audit every bf16 GEMM of a Depthformer v8 train step (diagnostic, GPU):
each mf.gemm call made under matmul_precision("bf16") is re-run in exact fp32 on operands
rounded to bf16 (the same descriptor), and the two results are compared -- they may differ
only by fp32 accumulation order.  Calls that differ by more than 1e-3 of the result's
magnitude are printed with their descriptor.
  python tools/bf16_audit.py [--full]     (--full: hidden 256, 480x640; default 64, 128x160)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402
from mdemi import functional as mf  # noqa: E402


def main():
    full = "--full" in sys.argv
    from mdemi.model.Depthformer import DepthformerV8
    from oracle.weights import closed_form_fill, rng_array
    if full:
        opt = {"hidden_dim": 256, "num_heads": 4, "num_bins": 256, "num_aux": 256, "img_size": [480, 640],
               "attn_drop_prob": 0.0, "drop_prob": 0.0}
        H, W = 480, 640
    else:
        opt = {"hidden_dim": 64, "num_heads": 4, "num_bins": 64, "num_aux": 32, "img_size": [128, 160],
               "attn_drop_prob": 0.0, "drop_prob": 0.0}
        H, W = 128, 160
    m = DepthformerV8.build(opt, 1e-3, 10.0)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    closed_form_fill(sd, seed=0.53, scale=0.03)
    m.load_state_dict(sd)
    m = m.cuda().train()
    img = torch.from_numpy(rng_array((2, 3, H, W), 84)).float().cuda()
    orig = mf.gemm
    bad, n = [], [0]

    def audited(A, B, C, M, N, K, **kw):
        if mf.get_matmul_precision() != "bf16" or kw.get("a_op", 0) or kw.get("b_op", 0):
            return orig(A, B, C, M, N, K, **kw)
        before = C.clone()
        out = orig(A, B, C, M, N, K, **kw)
        got = C.clone()
        C.copy_(before)
        kw2 = dict(kw)
        kw2["rowsum_a"] = None
        with mf.matmul_precision("fp32"):
            orig(A.to(torch.bfloat16).float(), B.to(torch.bfloat16).float(), C, M, N, K, **kw2)
        ref = C.clone()
        C.copy_(got)
        err = (got - ref).abs().max().item()
        mag = ref.abs().max().item()
        n[0] += 1
        desc = {k: v for k, v in kw.items() if not torch.is_tensor(v) and k != "conv"}
        if err > 1e-3 * mag + 1e-20:
            bad.append((err / (mag + 1e-30), M, N, K, desc))
        return out

    mf.gemm = audited
    try:
        with mf.matmul_precision("bf16"):
            depth, centers, attn = m(img)
            dy = torch.from_numpy(rng_array(tuple(depth.shape), 85)).float().cuda()
            (depth * dy).sum().backward()
        torch.cuda.synchronize()
    finally:
        mf.gemm = orig
    print(f"{n[0]} bf16 GEMM calls audited, {len(bad)} differ from the rounded-operand fp32 GEMM by > 1e-3")
    for b in sorted(bad, key=lambda r: -r[0])[:40]:
        print(f"  rel {b[0]:.3e}  M={b[1]} N={b[2]} K={b[3]}  {b[4]}")


if __name__ == "__main__":
    main()
