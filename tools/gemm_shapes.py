"""Per-shape GEMM timing inside one real train step of the bench workload: every libmdemi GEMM
call is bracketed by HIP events on its stream; calls are grouped by (layouts, ops, M, N, K,
batch, split) and printed by total time with their TFLOP/s, so the shapes that lose the most
time against the fp32 MFMA peak stand out.   python tools/gemm_shapes.py [--model newcrfs]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from mdemi import functional as mf  # noqa: E402


def main():
    import copy

    from mdemi.train import build_from_config
    args = bench.parse()
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[args.model]
    opt = copy.deepcopy(wl["opt"])
    B = args.batch or int(opt["dataloader"]["batch_size"])
    opt["dataloader"]["batch_size"] = B
    H, W = args.height or wl["h"], args.width or wl["w"]
    precision = args.precision or wl.get("precision", "fp32")
    torch.manual_seed(0)
    trainer = build_from_config(opt, device=dev, precision=precision)
    batches = [bench.synthetic_batch(B, H, W, dev, seed=1000 + i, data_type=opt["dataset"]["data_type"])
               for i in range(trainer.num_accum)]
    for _ in range(2):
        trainer.step(batches)
    torch.cuda.synchronize()
    recs = []
    orig = mf.gemm

    def timed(A, B, C, M, N, K, **kw):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(torch.cuda.current_stream())
        out = orig(A, B, C, M, N, K, **kw)
        e.record(torch.cuda.current_stream())
        split = kw.get("split_k")
        if split is None:
            split = mf._split_for(M, N, K)
        path = mf.LAST_GEMM[0]
        key = (kw.get("a_layout"), kw.get("b_layout"), kw.get("a_op", 0), M, N, K, kw.get("batch", 1), split, path)
        recs.append((key, s, e, bench._gemm_alg_bytes(A, B, M, N, K, kw, ob=2.0 if path == "b16" else 4.0)))
        return out

    mf.gemm = timed
    try:
        trainer.step(batches)
        torch.cuda.synchronize()
    finally:
        mf.gemm = orig
    by = collections.defaultdict(lambda: [0.0, 0, 0.0])
    for key, s, e, nb in recs:
        by[key][0] += s.elapsed_time(e) * 1e-3
        by[key][1] += 1
        by[key][2] += nb
    tot_t = sum(v[0] for v in by.values())
    tot_f = sum(2.0 * k[3] * k[4] * k[5] * k[6] * v[1] for k, v in by.items())
    print(f"{len(recs)} GEMM calls, {tot_t * 1e3:.2f} ms, {tot_f / tot_t / 1e12:.1f} TF/s")
    rows = []
    for k, (t, n, nb) in by.items():
        fl = 2.0 * k[3] * k[4] * k[5] * k[6] * n
        peak = 2500e12 if k[8] in ("b16", "bf16") else 157.3e12
        lost = t - max(fl / peak, nb / 8e12)  # time above the tighter of the MFMA and HBM floors
        rows.append((lost, k, t, n, fl / t / 1e12, nb / t / 1e9))
    rows.sort(reverse=True)
    print("lost_ms  time_ms calls  us/call   TF/s   GB/s  (a_layout,b_layout,a_op,M,N,K,batch,split,path)")
    for lost, k, t, n, tf, gbs in rows[:int(os.environ.get("SHAPES_TOP", "60"))]:
        print(f"{lost * 1e3:7.2f} {t * 1e3:8.2f} {n:5d} {t / n * 1e6:8.1f} {tf:6.1f} {gbs:6.0f}  {k}")


if __name__ == "__main__":
    main()
