"""Window-attention kernel timing on the NewCRFs-L07 480x640 bs=8 Swin stages
(fwd and fwd+bwd through the autograd op).  Prints one JSON line (ms)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402
from mdemi import functional as mf  # noqa: E402
from gemm_bench import bench  # noqa: E402


def main():
    L.load()
    out = {}
    for st, (H, W, C) in enumerate([(120, 160, 192), (60, 80, 384), (30, 40, 768), (15, 20, 1536)]):
        B, heads = 8, C // 32
        qkv = torch.randn(B * H * W, 3 * C, device="cuda").requires_grad_()
        bias = torch.randn(3 * C, device="cuda").requires_grad_()
        rpb = torch.randn(169, heads, device="cuda").requires_grad_()
        for shift in (0, 3):
            f = lambda: mf.window_attention(qkv, bias, qkv, bias, rpb, B, H, W, heads, 7, shift, 32 ** -0.5, C,
                                            v_off=2 * C)
            y = f()
            dy = torch.randn_like(y)
            out[f"s{st}_sh{shift}_fwd"] = round(bench(lambda: f()) * 1e3, 3)
            out[f"s{st}_sh{shift}_fwdbwd"] = round(bench(lambda: f().backward(dy)) * 1e3, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
