"""GEMM micro-benchmark on the NewCRFs-L07 train-step shapes (480x640, bs=8).
Times libmdemi's gemm_f32 per (layout, shape) with HIP events and prints
TFLOP/s.  MDEMI_LIB=<path> selects a library build (A/B of kernel variants)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402
from mdemi import functional as mf  # noqa: E402

B = 8
# (name, M, N, K): stage tokens at 480x640: 19200/4800/1200/300 per image
SHAPES = []
for st, (toks, C) in enumerate([(19200, 192), (4800, 384), (1200, 768), (300, 1536)]):
    M = B * toks
    SHAPES += [(f"s{st}_qkv", M, 3 * C, C), (f"s{st}_fc1", M, 4 * C, C), (f"s{st}_fc2", M, C, 4 * C)]


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    lib = L.load()
    variants = [(int(a), int(b)) for a, b in (v.split(":") for v in os.environ.get("VARIANTS", "0:0").split(","))]
    for v, gm in variants:
        lib.mdemi_gemm_set_variant(v, gm)
        run(f"v{v}g{gm}")


def run(tag):
    dev = "cuda"
    out = {}
    tot_fl = tot_t = 0.0
    for name, M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.05
        dy = torch.randn(M, N, device=dev)
        y = torch.empty(M, N, device=dev)
        dx = torch.empty(M, K, device=dev)
        dw = torch.empty(N, K, device=dev)
        cases = {
            "fwd": lambda: mf.gemm(x, w, y, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG,
                                   b_layout=L.L_KCONTIG, split_k=1),
            "dgrad": lambda: mf.gemm(dy, w, dx, M, K, N, lda=N, ldb=K, ldc=K, a_layout=L.L_KCONTIG,
                                     b_layout=L.L_MNCONTIG),
            "wgrad": lambda: mf.gemm(dy, x, dw, N, K, M, lda=N, ldb=K, ldc=K, a_layout=L.L_MNCONTIG,
                                     b_layout=L.L_MNCONTIG),
        }
        for cname, fn in cases.items():
            t = bench(fn)
            fl = 2.0 * M * N * K
            tot_fl += fl
            tot_t += t
            out[f"{name}.{cname}"] = round(fl / t / 1e12, 1)
    out["ALL"] = round(tot_fl / tot_t / 1e12, 2)
    out["variant"] = tag
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
