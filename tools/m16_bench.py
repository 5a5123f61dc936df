"""16-bit GEMM family micro-benchmark: one Linear fwd / dgrad / wgrad shape set of the
NeW-CRFs-L07 train step (480x640, bs 8) through mdemi.functional.gemm in each precision
(fp32 exact-product, fp32e three-plane bf16, bf16) and 16-bit variant; HIP-event timing,
TFLOP/s against each mode's MFMA peak.   python tools/m16_bench.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402
from mdemi import functional as mf  # noqa: E402

PEAK = {"fp32": 157.3, "fp32e": 2500.0 / 6, "bf16": 2500.0}
B = 8
SHAPES = [("s0_fc1 fwd", "kk", B * 19200, 768, 192), ("s2_fc2 fwd", "kk", B * 1200, 768, 3072),
          ("s2_fc1 dgrad", "kmn", B * 1200, 768, 3072), ("s1_fc1 wgrad", "mnmn", 1536, 384, B * 4800),
          ("s2_qkv wgrad", "mnmn", 2304, 768, B * 1200)]


def timeit(fn, iters):
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
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lib = L.load()
    dev = "cuda"
    kk_only = os.environ.get("M16_KK_ONLY") == "1"  # study builds (tools/m16_study.sh -DMDEMI_M16_KK_ONLY)
    for name, kind, M, N, K in SHAPES:
        if kk_only and kind != "kk":
            continue
        if kind == "kk":  # C[M,N] = A[M,K] B[N,K]^T
            A, Bm = torch.randn(M, K, device=dev), torch.randn(N, K, device=dev)
            kw = dict(lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG)
        elif kind == "kmn":  # C[M,N] = A[M,K] B[K,N]
            A, Bm = torch.randn(M, K, device=dev), torch.randn(K, N, device=dev)
            kw = dict(lda=K, ldb=N, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG)
        else:  # C[M,N] = A[K,M]^T B[K,N]
            A, Bm = torch.randn(K, M, device=dev), torch.randn(K, N, device=dev)
            kw = dict(lda=M, ldb=N, ldc=N, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG)
        C = torch.empty(M, N, device=dev)
        fl = 2.0 * M * N * K
        row = []
        for prec, variants in (("fp32", [-1]), ("fp32e", [0, 1, 2]), ("bf16", [0, 1, 2])):
            for v in variants:
                if prec != "fp32":
                    lib.mdemi_gemm_set_variant_m16(v)
                with mf.matmul_precision(prec):
                    t = timeit(lambda: mf.gemm(A, Bm, C, M, N, K, **kw), iters)
                tf = fl / t / 1e12
                row.append(f"{prec}{'' if v < 0 else '/v' + str(v)} {tf:7.1f} TF ({tf / PEAK[prec]:.2f})")
        lib.mdemi_gemm_set_variant_m16(-1)
        print(f"{name:14s} M={M:6d} N={N:5d} K={K:6d} | " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
