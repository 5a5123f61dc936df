"""Depthwise conv kernels (csrc/effnet.hip) at the EfficientNet-B5 stride-1 shapes of the
configs[4] / AdaBins steps (NYU 480x640, batch 8): forward, input gradient and weight gradient
(partials + column sum) per shape, as hipGraphs of back-to-back launches, with the achieved
GB/s of each (algorithmic bytes: 8 B per output element forward / input gradient, 8 B per
output element for the weight gradient's two reads).  Also checks the three outputs against
torch's fp64 depthwise conv.
   MDEMI_DW_TY=1|2|4 python tools/dw_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mdemi import _lib as L  # noqa: E402

REPS = 10


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


def main():
    lib = L.load()
    n = 8
    tot = [0.0, 0.0, 0.0]
    for (h, w, c, k, cnt) in ((240, 320, 48, 3, 1), (240, 320, 24, 3, 2), (120, 160, 240, 3, 4), (60, 80, 384, 5, 4),
                              (30, 40, 768, 3, 6), (30, 40, 1056, 5, 6), (15, 20, 1824, 5, 8), (15, 20, 3072, 3, 2)):
        g = torch.Generator(device="cpu").manual_seed(h * c + k)
        x = torch.randn(n, h, w, c, generator=g).cuda()
        wt = (torch.randn(c, 1, k, k, generator=g) * 0.3).cuda()
        dy = torch.randn(n, h, w, c, generator=g).cuda()
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        dw = torch.empty_like(wt)
        p = k // 2
        ws = torch.empty(lib.mdemi_dwconv_bwd_workspace_size(n, c, k, h, w), dtype=torch.uint8, device="cuda")

        def fwd():
            L.check(lib.mdemi_dwconv_fwd(x.data_ptr(), wt.data_ptr(), y.data_ptr(), n, h, w, c, k, 1, p, p, h, w, L.stream()),
                    "dwconv_fwd")

        def bwd_dx():
            L.check(lib.mdemi_dwconv_bwd(dy.data_ptr(), x.data_ptr(), wt.data_ptr(), dx.data_ptr(), None, n, h, w, c, k,
                                         1, p, p, h, w, ws.data_ptr(), L.stream()), "dwconv_bwd")

        def bwd_dw():
            L.check(lib.mdemi_dwconv_bwd(dy.data_ptr(), x.data_ptr(), wt.data_ptr(), None, dw.data_ptr(), n, h, w, c, k,
                                         1, p, p, h, w, ws.data_ptr(), L.stream()), "dwconv_bwd")

        tf, tx, tw = graph_time(fwd), graph_time(bwd_dx), graph_time(bwd_dw)
        # check against fp64 torch (NCHW)
        xr = x.double().permute(0, 3, 1, 2).requires_grad_()
        wr = wt.double().requires_grad_()
        yr = F.conv2d(xr, wr, padding=p, groups=c)
        yr.backward(dy.double().permute(0, 3, 1, 2))
        ey = ((y.double().permute(0, 3, 1, 2) - yr).abs().max() / yr.abs().max()).item()
        ex = ((dx.double().permute(0, 3, 1, 2) - xr.grad).abs().max() / xr.grad.abs().max()).item()
        ew = ((dw.double() - wr.grad).abs().max() / wr.grad.abs().max()).item()
        nb = 8.0 * x.numel()
        for i, t in enumerate((tf, tx, tw)):
            tot[i] += cnt * t
        print(f"k{k} {h}x{w}x{c:5d} (x{cnt}): fwd {tf * 1e6:7.1f} us {nb / tf / 1e9:6.0f} GB/s   dx {tx * 1e6:7.1f} us "
              f"{nb / tx / 1e9:6.0f} GB/s   dw {tw * 1e6:7.1f} us {nb / tw / 1e9:6.0f} GB/s   rel err {ey:.1e} "
              f"{ex:.1e} {ew:.1e}", flush=True)
        assert ey < 1e-5 and ex < 1e-5 and ew < 1e-4, (ey, ex, ew)
    print(f"MDEMI_DW_TY={os.environ.get('MDEMI_DW_TY', '4')}: per configs[4] step (stride-1 blocks): fwd "
          f"{tot[0] * 1e3:.3f} ms, dx {tot[1] * 1e3:.3f} ms, dw {tot[2] * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
