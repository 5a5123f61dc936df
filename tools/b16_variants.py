"""Every bf16-operand GEMM variant (gemm_b16_kernel.h: 0 128-row, 1 256-row, 2 two K tiles per
stage) on the configs[4] shapes that lose the most time
(Depthformer v8 bf16, NYU 480x640, batch 8: profiles/round6/), at several split-K factors.
Each point is a hipGraph of 20 back-to-back launches, so no host launch gap is timed.
   python tools/b16_variants.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402
from mdemi import functional as mf  # noqa: E402

REPS = 20


def graph_time(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * REPS) * 1e-3


def case(lib, name, M, N, K, al, bl, a_shape, b_shape, c_shape, splits, variants=(0, 1, 2), **kw):
    A16 = torch.randn(*a_shape, device="cuda").to(torch.bfloat16)
    B16 = (torch.randn(*b_shape, device="cuda") * 0.05).to(torch.bfloat16)
    C = torch.empty(*c_shape, device="cuda")
    ref = None
    nbytes = 2.0 * (A16.numel() + B16.numel()) + 4.0 * C.numel()
    for s in splits:
        row = []
        for v in variants:
            assert lib.mdemi_gemm_set_variant_b16(v) == 0
            try:
                with mf.matmul_precision("bf16"):
                    fn = lambda: mf.gemm(None, None, C, M, N, K, a_layout=al, b_layout=bl, a16=A16, b16=B16,  # noqa: E731
                                         split_k=s, **kw)
                    fn()
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = C.clone()
                    elif s == splits[0]:
                        assert torch.equal(C, ref), (name, s, v)  # same k order: bit-identical
                    t = graph_time(fn)
            finally:
                lib.mdemi_gemm_set_variant_b16(-1)
            row.append(f"v{v} {t * 1e6:7.1f}")
        print(f"{name:30s} M={M:6d} N={N:5d} K={K:7d} split {s:3d}: " + "  ".join(row) +
              f"   (bytes at 5 TB/s {nbytes / 5e12 * 1e6:.1f} us)", flush=True)


def main():
    lib = L.load()
    torch.manual_seed(0)
    KC, MN = L.L_KCONTIG, L.L_MNCONTIG
    n = 8
    # EfficientNet 1x1 convs of the 15x20 / 30x40 stages: forward, data and weight gradients
    for (hh, ww, ci, cx) in ((15, 20, 304, 1824), (30, 40, 176, 1056), (30, 40, 128, 768), (15, 20, 512, 3072)):
        M = n * hh * ww
        case(lib, f"1x1 fwd {hh}x{ww} {cx}->{ci}", M, ci, cx, KC, KC, (M, cx), (ci, cx), (M, ci), (1, 2, 4, 8),
             lda=cx, ldb=cx, ldc=ci)
        case(lib, f"1x1 fwd {hh}x{ww} {ci}->{cx}", M, cx, ci, KC, KC, (M, ci), (cx, ci), (M, cx), (1, 2),
             lda=ci, ldb=ci, ldc=cx)
        case(lib, f"1x1 dgrad {hh}x{ww} {cx}->{ci}", M, ci, cx, KC, MN, (M, cx), (cx, ci), (M, ci), (1, 2, 4, 7),
             lda=cx, ldb=ci, ldc=ci)
        case(lib, f"1x1 wgrad {hh}x{ww} {cx}x{ci}", cx, ci, M, MN, MN, (M, cx), (M, ci), (cx, ci), (1, 2, 4, 9),
             lda=cx, ldb=ci, ldc=ci)
    # a full-chip shape for reference: 1x1 expand at 120x160
    M = n * 120 * 160
    case(lib, "1x1 fwd 120x160 40->240", M, 240, 40, KC, KC, (M, 40), (240, 40), (M, 240), (1,),
         lda=40, ldb=40, ldc=240)
    case(lib, "1x1 wgrad 120x160 240x40", 240, 40, M, MN, MN, (M, 240), (M, 40), (240, 40), (64, 256, 512),
         lda=240, ldb=40, ldc=40)
    # decoder 3x3 conv at 240x320 (the largest GEMMs of the step)
    h, w, c = 240, 320, 256
    g = mf._geom(n, h, w, c, h, w, 3, 3, 1, 1, L.PAD_REPLICATE)
    M = n * h * w
    case(lib, "conv3x3 fwd 240x320 256->256", M, c, 9 * c, L.L_CONV, KC, (n, h, w, c), (c, 9 * c), (n, h, w, c),
         (1,), lda=0, ldb=9 * c, ldc=c, conv=g)


if __name__ == "__main__":
    main()
