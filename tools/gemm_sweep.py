"""GEMM shape sweep (fwd layout KCONTIG x KCONTIG): TFLOP/s vs M, N, K to
separate kernel-intrinsic limits from shape effects.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402
from mdemi import functional as mf  # noqa: E402
from gemm_bench import bench  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 8192, 1024), (153600, 768, 192), (153600, 768, 384), (153600, 768, 768),
          (153600, 768, 1536), (153600, 192, 768), (38400, 1536, 384), (9600, 3072, 768), (153600, 1536, 192)]


def main():
    L.load()
    out = {}
    for M, N, K in [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]] or SHAPES:
        a = torch.randn(M, K, device="cuda")
        b = torch.randn(N, K, device="cuda")
        c = torch.empty(M, N, device="cuda")
        t = bench(lambda: mf.gemm(a, b, c, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG,
                                  b_layout=L.L_KCONTIG, split_k=1))
        out[f"{M}x{N}x{K}"] = round(2.0 * M * N * K / t / 1e12, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
