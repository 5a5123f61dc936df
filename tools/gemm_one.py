"""Run one GEMM shape with a fixed pipelining variant a few times (for rocprofv3 --pmc passes):
  python tools/gemm_one.py M N K variant [layouts=fwd|dgrad|wgrad] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402
from mdemi import functional as mf  # noqa: E402

M, N, K, v = (int(a) for a in sys.argv[1:5])
lay = sys.argv[5] if len(sys.argv) > 5 else "fwd"
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
lib = L.load()
lib.mdemi_gemm_set_variant(v, 8)
a = torch.randn(M, K, device="cuda")
b = torch.randn(N, K, device="cuda")
c = torch.empty(M, N, device="cuda")
dy, x = torch.randn(K, M, device="cuda"), torch.randn(K, N, device="cuda")
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for i in range(reps + 2):
    if i == 2:
        s.record()
    if lay == "fwd":
        mf.gemm(a, b, c, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, split_k=1)
    elif lay == "dgrad":
        mf.gemm(a, b.t().contiguous() if i == 0 else bt, c, M, N, K, lda=K, ldb=N, ldc=N, a_layout=L.L_KCONTIG,
                b_layout=L.L_MNCONTIG, split_k=1)
        bt = b.t().contiguous()
    else:
        mf.gemm(dy, x, c, M, N, K, lda=M, ldb=N, ldc=N, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG, split_k=1)
e.record()
torch.cuda.synchronize()
t = s.elapsed_time(e) / reps * 1e-3
print(f"M={M} N={N} K={K} v={v} {lay}: {t * 1e6:.1f} us  {2.0 * M * N * K / t / 1e12:.1f} TF/s", flush=True)
