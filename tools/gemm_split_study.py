"""Split-K study on the train-step shapes that the heuristic splits: time (GEMM + reduce) per
split factor, autotuned variant.   python tools/gemm_split_study.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402
from mdemi import functional as mf  # noqa: E402

# (layout, M, N, K) from profiles/r02_gemm_shapes.txt
SHAPES = [("wgrad", 3072, 768, 9600), ("wgrad", 2304, 768, 9600), ("wgrad", 768, 768, 9600),
          ("wgrad", 768, 3072, 9600), ("wgrad", 576, 192, 153600), ("wgrad", 768, 192, 153600),
          ("wgrad", 192, 768, 153600), ("wgrad", 384, 1536, 38400), ("wgrad", 1536, 384, 38400),
          ("wgrad", 192, 192, 153600), ("wgrad", 6144, 1536, 2400), ("dgrad", 2400, 1536, 6144)]
CANDIDATES = [int(v) for v in os.environ.get("SPLITS", "1,2,3,4,5,6,7,8,10,12,14,16,18,24,28,36").split(",")]


def run(lay, M, N, K, split):
    if lay == "dgrad":
        a, b = torch.randn(M, K, device="cuda"), torch.randn(K, N, device="cuda")
        fn = lambda c: mf.gemm(a, b, c, M, N, K, lda=K, ldb=N, ldc=N, a_layout=L.L_KCONTIG,  # noqa: E731
                               b_layout=L.L_MNCONTIG, split_k=split)
    else:
        a, b = torch.randn(K, M, device="cuda"), torch.randn(K, N, device="cuda")
        fn = lambda c: mf.gemm(a, b, c, M, N, K, lda=M, ldb=N, ldc=N, a_layout=L.L_MNCONTIG,  # noqa: E731
                               b_layout=L.L_MNCONTIG, split_k=split)
    c = torch.empty(M, N, device="cuda")
    for _ in range(3):
        fn(c)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        fn(c)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 10 * 1e3


for lay, M, N, K in SHAPES:
    cur = mf._split_for(M, N, K)
    kt = -(-K // 16)
    res = {sp: run(lay, M, N, K, sp) for sp in sorted({cur, *CANDIDATES, 2 * cur, 3 * cur}) if sp <= max(1, kt // 8)}
    best = min(res, key=res.get)
    print(f"{lay} {M}x{N}x{K} tiles {-(-M // 128) * -(-N // 128)} heuristic split {cur} ({res[cur]:.0f}us): "
          + " ".join(f"s{k}={v:.0f}" for k, v in res.items()) + f"  best s{best} ({res[best]:.0f}us)", flush=True)
