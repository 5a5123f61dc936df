"""Training-mode BatchNorm (+SiLU) sweeps at the EfficientNet-B5 shapes of configs[4]
(Depthformer v8, NYU 480x640, batch 8): per call the forward (mdemi_bn_train_fwd16 with the
bf16 output copy) and backward (mdemi_chnorm_bwd16 with the bf16 input-gradient copy) time
and the fraction of HBM peak their algorithmic bytes reach.
  forward : statistics (sum x, sum x^2: one read) 4 B + apply (4 B in, 4 + 2 B out)
  backward: partial(x, dy) 8 B + apply (x, dy in; dx 4 B + dx16 2 B out)
per element.  python tools/bn_bench.py  (run under rocprofv3 --kernel-trace --stats for the
per-kernel split)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402

from mdemi import _lib as L  # noqa: E402

HBM = 8000.0  # GB/s
# (rows = batch * H * W, channels): MBConv expand / depthwise maps of tf_efficientnet_b5 at 480x640
SHAPES = [(614400, 144), (153600, 144), (153600, 240), (38400, 240), (38400, 384), (9600, 384), (9600, 768),
          (9600, 1056), (2400, 1056), (2400, 1824), (2400, 3072), (614400, 48), (614400, 24)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    lib = L.load()
    torch.manual_seed(0)
    tot = [0.0, 0.0, 0.0, 0.0]
    for rows, c in SHAPES:
        n, hw = 8, rows // 8
        x = torch.randn(rows, c, device="cuda") * 2 + 0.5
        dy = torch.randn(rows, c, device="cuda")
        g = torch.rand(c, device="cuda") + 0.5
        b = torch.randn(c, device="cuda") * 0.1
        y, dx = torch.empty_like(x), torch.empty_like(x)
        y16 = torch.empty(rows, c, device="cuda", dtype=torch.bfloat16)
        dx16 = torch.empty_like(y16)
        mean, rstd = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
        rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
        dg, db = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
        ws = torch.empty(lib.mdemi_chnorm_workspace_size(n, hw, c, c, 1) // 4 + 1, device="cuda")
        fwd = lambda: L.check(lib.mdemi_bn_train_fwd16(  # noqa: E731
            x.data_ptr(), g.data_ptr(), b.data_ptr(), y.data_ptr(), y16.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
            rm.data_ptr(), rv.data_ptr(), None, 0.1, n, hw, c, 1e-3, L.ACT_SILU, ws.data_ptr(), L.stream()), "fwd")
        bwd = lambda: L.check(lib.mdemi_chnorm_bwd16(  # noqa: E731
            dy.data_ptr(), x.data_ptr(), None, mean.data_ptr(), rstd.data_ptr(), g.data_ptr(), b.data_ptr(),
            dx.data_ptr(), dx16.data_ptr(), dg.data_ptr(), db.data_ptr(), n, hw, c, c, 1, L.ACT_SILU, ws.data_ptr(),
            L.stream()), "bwd")
        tf, tb = timeit(fwd), timeit(bwd)
        e = rows * c
        bf, bb = e * (4 + 10), e * (8 + 14)
        tot[0] += tf; tot[1] += tb; tot[2] += bf; tot[3] += bb
        print(f"rows={rows:7d} C={c:5d}  fwd {tf * 1e6:8.1f} us ({bf / tf / 1e9 / HBM:.2f} of HBM)   "
              f"bwd {tb * 1e6:8.1f} us ({bb / tb / 1e9 / HBM:.2f} of HBM)", flush=True)
    print(f"all shapes: fwd {tot[0] * 1e6:.1f} us ({tot[2] / tot[0] / 1e9 / HBM:.2f})  "
          f"bwd {tot[1] * 1e6:.1f} us ({tot[3] / tot[1] / 1e9 / HBM:.2f})")


if __name__ == "__main__":
    main()
