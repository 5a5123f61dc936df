"""Time the fp32 GEMM family per pipelining variant on a few model shapes (one process, one library):
  MDEMI_LIB=tools/study/<tag>/libmdemi.so python tools/gemm_study.py <tag> [variants=0,1,3,4,5,6,7]
Prints one line per (shape, variant) with µs and TF/s (HIP events, 10 reps after 2 warm-ups)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402
from mdemi import functional as mf  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
variants = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1,3,4,5,6,7").split(",")]
shapes = os.environ.get("SHAPES", "9600x3072x768:fwd,9600x768x3072:fwd,9600x768x3072:dgrad,3072x768x9600:wgrad")
lib = L.load()
for spec in shapes.split(","):
    dims, lay = spec.split(":")
    M, N, K = (int(x) for x in dims.split("x"))
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda")
    bk = torch.randn(N, K, device="cuda")
    bn = torch.randn(K, N, device="cuda")
    am = torch.randn(K, M, device="cuda")
    c = torch.empty(M, N, device="cuda")

    def run():
        if lay == "fwd":
            mf.gemm(a, bk, c, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, split_k=1)
        elif lay == "dgrad":
            mf.gemm(a, bn, c, M, N, K, lda=K, ldb=N, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG, split_k=1)
        else:
            mf.gemm(am, bn, c, M, N, K, lda=M, ldb=N, ldc=N, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
                    split_k=1)

    for v in variants:
        lib.mdemi_gemm_set_variant(v, 8)
        for _ in range(2):
            run()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            run()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / 10 * 1e-3
        print(f"{tag} {lay} M={M} N={N} K={K} v={v}: {t * 1e6:8.1f} us {2.0 * M * N * K / t / 1e12:6.1f} TF/s",
              flush=True)
