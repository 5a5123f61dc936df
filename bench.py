#!/usr/bin/env python3
"""Throughput benchmark of the dense-depth train step on MI355X.

metric (BASELINE.json): images/sec (train step) NYU 640x480 bs=8/GPU.
Default workload: NeW-CRFs Swin-L (large07) train step at NYU 480x640, batch 8
per GPU — the reference config json/nyu/newcrfs/newcrfs_github_eval.json
(batch_size 8, loss alpha 10 / beta 0.15, AdamW lr 2e-5 wd 0, grad_norm 0.1).
A step = forward + SILog loss + backward + clip + AdamW update (+ the RCCL
gradient all-reduce when N > 1), all on libmdemi kernels; synthetic inputs
(SURVEY §8d): ImageNet-normalised uniform images, NYU-style depth U(0.5, 10)
inside the [45:472, 43:608] valid region.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU)

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix peak (v_mfma_f32_32x32x2_f32)
HBM_PEAK_GBS = 8000.0

WORKLOADS = {
    "newcrfs": dict(model="NewCRFs-L07", h=480, w=640, batch=8, max_depth=10.0,
                    workload="NewCRFs Swin-L (large07) train step, NYU 480x640",
                    ref_cfg="json/nyu/newcrfs/newcrfs_github_eval.json"),
    # BASELINE.json configs[2] / north_star target shape
    "newcrfs_kitti": dict(model="NewCRFs-L07", h=352, w=1216, batch=8, max_depth=80.0,
                          workload="NewCRFs Swin-L (large07) train step, KITTI 352x1216",
                          ref_cfg="json/kitti/newcrfs/newcrfs_github_eval.json"),
    # BASELINE.json configs[1]: AdaBins (EfficientNet-B5 + DecoderBN + mViT + bin head), NYU bs=16;
    # json/nyu/adabins/adabins_cham_per_batch.json: AdamW lr 3.57e-4 wd 0.1, grad_norm 0.1, SILog a10 b0.15
    # + its chamfer bin loss (loss.chamfer_weight 0.1) on the bin edges
    "adabins": dict(model="AdaBins-B5", h=480, w=640, batch=16, max_depth=10.0, lr=3.57e-4, wd=0.1, beta=0.15,
                    per_image=False, chamfer=0.1, workload="AdaBins EfficientNet-B5 train step, NYU 480x640",
                    ref_cfg="json/nyu/adabins/adabins_cham_per_batch.json"),
    # Depthformer v8 (json/kitti/depthformer/depthformer_v8_cham_loss_per_image_4gpu.json model/optimizer
    # block: hidden 256, 4 heads, 256 bins / aux tokens, lr 3.2e-4 wd 0.1, SILog a10 b0.5 per image,
    # chamfer 0.1 on the bin centres) at the
    # NYU crop, fp32 (BASELINE configs[4]'s bf16 + hipGraph variant is not built)
    "depthformer": dict(model="DepthformerV8-B5", h=480, w=640, batch=8, max_depth=10.0, lr=3.2e-4, wd=0.1,
                        beta=0.5, per_image=True, chamfer=0.1, workload="Depthformer v8 train step, NYU 480x640 (fp32)",
                        ref_cfg="json/kitti/depthformer/depthformer_v8_cham_loss_per_image_4gpu.json"),
}
DFV8_OPT = {"hidden_dim": 256, "num_heads": 4, "num_bins": 256, "num_aux": 256, "img_size": [480, 640],
            "attn_drop_prob": 0.1, "drop_prob": 0.2}
# HBM bytes per launch of the roofline kernel family, from the committed
# rocprofv3 --pmc passes (tools/pmc_traffic.py; FETCH_SIZE doubled per the
# gfx950 correction).  None when no profile matches the kernel.
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="newcrfs", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=15.0)
    ap.add_argument("--no-roofline", action="store_true")
    return ap.parse_args()


def synthetic_batch(B, H, W, device, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    img = torch.rand(B, 3, H, W, generator=g)
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    img = (img - mean) / std  # depth_dataset.py:290 (ImageNet Normalize)
    gt = torch.rand(B, 1, H, W, generator=g) * 9.5 + 0.5
    valid = torch.zeros(B, 1, H, W)
    valid[:, :, 45 * H // 480:472 * H // 480, 43 * W // 640:608 * W // 640] = 1  # NYU valid region
    gt = gt * valid
    return img.to(device), gt.to(device)


def build(args, device):
    from mdemi.train import FusedAdamW, SILogLoss
    cfg = WORKLOADS[args.model]
    torch.manual_seed(0)
    if args.model == "adabins":
        from mdemi.model.Adabins import UnetAdaptiveBins
        model = UnetAdaptiveBins.build(256, 1e-3, cfg["max_depth"])
    elif args.model == "depthformer":
        from mdemi.model.Depthformer import DepthformerV8
        model = DepthformerV8.build(DFV8_OPT, 1e-3, cfg["max_depth"])
    else:
        from mdemi.model.NewCRFs import NewCRFDepth
        model = NewCRFDepth(version="large07", inv_depth=False, max_depth=cfg["max_depth"])
    model = model.to(device).train()
    opt = FusedAdamW(model.parameters(), lr=cfg.get("lr", 2e-5), weight_decay=cfg.get("wd", 0.0), max_grad_norm=0.1)
    silog = SILogLoss(alpha=10.0, beta=cfg.get("beta", 0.15), per_image=cfg.get("per_image", False), min_depth=1e-3)
    return model, opt, TrainLoss(silog, cfg.get("chamfer", 0.0), from_edges=(args.model == "adabins"))


class TrainLoss:
    """SILog on the depth (+ chamfer_weight x the bin chamfer loss on AdaBins' edges / Depthformer's
    centres when the config sets loss.chamfer_weight)."""

    def __init__(self, silog, chamfer_weight, from_edges):
        from mdemi.train import BinsChamferLoss
        self.silog, self.w = silog, float(chamfer_weight)
        self.chamfer = BinsChamferLoss(1e-3, from_edges=from_edges) if self.w > 0 else None

    def __call__(self, out, gt):
        pred = out[0] if isinstance(out, tuple) else out  # AdaBins / Depthformer: (depth at H/2, bins, ...)
        loss = self.silog(pred, gt)  # SILogLoss upsamples a half-resolution prediction to the GT first
        if self.chamfer is not None:
            loss = loss + self.w * self.chamfer(out[1], gt)
        return loss


def train_step(model, opt, loss_fn, img, gt, ddp=None):
    loss = loss_fn(model(img), gt)
    loss.backward()
    if ddp is not None:
        ddp.finish()
    opt.step()
    opt.zero_grad(set_to_none=True)
    return loss


def gemm_roofline(model, opt, loss_fn, img, gt, ddp):
    """One instrumented step: HIP events around every libmdemi GEMM launch on its stream;
    algorithmic FLOPs (2*M*N*K per GEMM) / measured kernel time, grouped by kernel."""
    from mdemi import functional as mf
    recs = []
    orig = mf.gemm

    def timed(A, B, C, M, N, K, **kw):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(torch.cuda.current_stream())
        out = orig(A, B, C, M, N, K, **kw)
        e.record(torch.cuda.current_stream())
        key = (kw.get("a_layout"), kw.get("b_layout"), kw.get("a_op", 0), kw.get("b_op", 0))
        recs.append((key, 2.0 * M * N * K * kw.get("batch", 1), s, e))
        return out

    mf.gemm = timed
    try:
        train_step(model, opt, loss_fn, img, gt, ddp)
        torch.cuda.synchronize()
    finally:
        mf.gemm = orig
    by = {}
    for key, fl, s, e in recs:
        t = s.elapsed_time(e) * 1e-3
        a = by.setdefault(key, [0.0, 0.0, 0])
        a[0] += fl
        a[1] += t
        a[2] += 1
    tot_fl = sum(v[0] for v in by.values())
    tot_t = sum(v[1] for v in by.values())
    dom = max(by.items(), key=lambda kv: kv[1][1])
    return by, dom, tot_fl, tot_t


KERNEL_NAME = {0: "KCONTIG", 1: "MNCONTIG", 2: "CONV"}


def profiled_traffic(regex, workload):
    try:
        with open(TRAFFIC_FILE) as f:
            prof = json.load(f)
    except (OSError, ValueError):
        return None
    fam = prof.get(workload, {}).get("families", {}).get(regex)
    return None if fam is None else fam.get("traffic_bytes_per_launch")


def cpu_baseline(model, name, H, W, budget_s):
    """The oracle (CPU restatement of the reference path: oracle/newcrfs.py, oracle/adabins.py,
    oracle/depthformer.py) timed on the host cores: fp32 forward + SILog + backward + clipped AdamW
    step at batch 1, same weights."""
    from oracle import metrics as omet
    cfg = WORKLOADS[name]
    threads = torch.get_num_threads()
    P = {k: v.detach().float().cpu().clone().requires_grad_(torch.is_floating_point(v))
         for k, v in model.state_dict().items()}
    params = [v for v in P.values() if v.requires_grad]
    opt = torch.optim.AdamW(params, lr=cfg.get("lr", 2e-5), weight_decay=cfg.get("wd", 0.0))
    img, gt = synthetic_batch(1, H, W, "cpu", seed=1)
    if name == "adabins":
        from oracle import adabins as oab
        fwd = lambda: oab.unet_adaptive_bins(P, img, 1e-3, cfg["max_depth"])  # noqa: E731
    elif name == "depthformer":
        from oracle import depthformer as odf
        opt_m = dict(DFV8_OPT, attn_drop_prob=0.0, drop_prob=0.0)
        fwd = lambda: odf.depthformer_v8_full(P, img, opt_m, 1e-3, cfg["max_depth"])  # noqa: E731
    else:
        from oracle import newcrfs as onc
        fwd = lambda: onc.newcrf_depth(P, img, "large07", max_depth=cfg["max_depth"])  # noqa: E731

    def step():
        out = fwd()
        pred = out[0] if isinstance(out, tuple) else out
        if pred.shape[-2:] != gt.shape[-2:]:
            pred = torch.nn.functional.interpolate(pred, gt.shape[-2:], mode="bilinear", align_corners=True)
        loss = omet.silog_loss(pred, gt, 1e-3, 10.0, cfg.get("beta", 0.15), cfg.get("per_image", False))
        if cfg.get("chamfer", 0.0) > 0:
            from oracle.adabins import bins_chamfer_loss
            loss = loss + cfg["chamfer"] * bins_chamfer_loss(out[1], gt, 1e-3, from_edges=(name == "adabins"))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 0.1)
        opt.step()
        opt.zero_grad(set_to_none=True)

    t0 = time.perf_counter()
    step()  # warm-up
    first = time.perf_counter() - t0
    n = max(1, min(5, int(budget_s / max(first, 1e-3))))
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    dt = (time.perf_counter() - t0) / n
    return {"value": round(1.0 / dt, 4), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"oracle {cfg['model']} fp32 train step (fwd+SILog{'+chamfer' if cfg.get('chamfer') else ''}+bwd+AdamW), batch 1 at {H}x{W}, "
                      f"{n} timed steps after 1 warm-up, {threads} threads, {os.cpu_count()} host CPUs visible"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    cfg = WORKLOADS[args.model]
    B = args.batch or cfg["batch"]
    H = args.height or cfg["h"]
    W = args.width or cfg["w"]

    model, opt, loss_fn = build(args, device)
    ddp = None
    if world > 1:  # bucketed RCCL gradient mean overlapped with backward (mdemi/train/ddp.py)
        from mdemi.train import GradAllReduce, broadcast_parameters
        broadcast_parameters(model)  # identical replicas (DDP broadcasts rank 0's weights)
        ddp = GradAllReduce(model, bucket_mb=64.0)
    img, gt = synthetic_batch(B, H, W, device, seed=1000 + rank)

    for _ in range(args.warmup):
        train_step(model, opt, loss_fn, img, gt, ddp)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = train_step(model, opt, loss_fn, img, gt, ddp)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    loss_v = float(loss.item())
    ms = elapsed / args.steps * 1e3
    value = B * world * args.steps / elapsed

    roof = None
    extra = {}
    if not args.no_roofline:
        by, dom, tot_fl, tot_t = gemm_roofline(model, opt, loss_fn, img, gt, ddp)
        (al, bl, aop, bop), (fl, t, cnt) = dom
        ach = fl / t / 1e12
        regex = f"gemm_f32_kernel<{al}, {bl}, {aop}, {bop},"
        roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                "traffic": profiled_traffic(regex, args.model), "traffic_unit": "HBM bytes/launch (rocprofv3 PMC)",
                "kernel": f"gemm_f32_kernel<{KERNEL_NAME[al]},{KERNEL_NAME[bl]},{aop},{bop}> (all pipelining variants)",
                "kernel_regex": regex, "launches": cnt, "avg_launch_us": round(t / cnt * 1e6, 2),
                "flops_per_launch": fl / cnt}
        extra["gemm_all"] = {"achieved_tflops": round(tot_fl / tot_t / 1e12, 2), "gemm_ms_per_step": round(tot_t * 1e3, 2),
                             "gemm_tflop_per_step": round(tot_fl / 1e12, 3),
                             "frac": round(tot_fl / tot_t / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)}
        extra["step_mfma_frac"] = round(tot_fl / (ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(model, args.model, H, W, args.cpu_budget_s)

    if rank == 0:
        line = {
            "metric": ("images/sec (train step) NYU 640x480 bs=8/GPU" if args.model == "newcrfs" else
                       f"images/sec (train step) {cfg['model']} {W}x{H} bs={B}/GPU"),
            "value": round(value, 3), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic (random-init weights)",
            "config": {"workload": cfg["workload"], "model": cfg["model"], "global_batch": B * world,
                       "per_gpu_batch": B, "image": [H, W], "parallelism": f"dp{world}",
                       "reference_config": cfg["ref_cfg"]},
            "roofline": roof, "cpu_baseline": cpu, "loss": round(loss_v, 5), **extra,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
