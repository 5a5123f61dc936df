#!/usr/bin/env python3
"""Throughput benchmark of the dense-depth train step on MI355X.

metric (BASELINE.json): images/sec (train step) NYU 640x480 bs=8/GPU.
Default workload: NeW-CRFs Swin-L (large07) train step at NYU 480x640, batch 8
per GPU, built from the reference config json/nyu/newcrfs/newcrfs_github_eval.json
by mdemi.train.build_from_config (the restated run.py construction): SILog
alpha 10 / beta 0.15, AdamW lr 2e-5 wd 0 with OneCycle, grad_norm 0.1.
A step = forward + loss + backward + (N > 1: bucketed RCCL gradient all-reduce
overlapped with the backward) + clipped AdamW update + scheduler step, all on
libmdemi kernels; synthetic inputs.  The same line carries a
secondary measurement at the north_star shape (NeW-CRFs KITTI 352x1216, bs 8/GPU;
BASELINE configs[2], and configs[3] when N = 8).

  python bench.py [--gpus N --steps K --warmup W]        (N > 1: starts N ranks itself)
  torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)
  python bench.py --config json/kitti/adabins/adabins_cham_per_batch_4gpu.json

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "monocular-depth-estimation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix peak (v_mfma_f32_32x32x2_f32)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense BF16 MFMA (no sparsity)
# fp32e = fp32 GEMM as six bf16-plane products per 32x32x16 block: the bf16 MFMA peak / 6
F32E_MFMA_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6.0
HBM_PEAK_GBS = 8000.0
CPU_SHARE_PER_GPU = 16  # the GPU box's host-CPU share per GPU (OMP_NUM_THREADS there)

# The reference configs that define each workload (the keys build_from_config reads; the
# reference tree is not on the GPU box, so they are restated here with their source).
_NEWCRFS_NYU = {  # json/nyu/newcrfs/newcrfs_github_eval.json
    "model": {"name": "newcrfs"}, "loss": {"alpha": 10.0, "beta": 0.15, "per_image": False},
    "dataset": {"data_type": "NYU"}, "dataloader": {"batch_size": 8},
    "optimizer": {"lr": 2e-5, "weight_decay": 0.0},
    "scheduler": {"name": "onecycle", "pct_start": 0.3, "div_factor": 25, "final_div_factor": 100},
    "train": {"epoch": 25, "num_accum": 1, "grad_norm": 0.1},
    "eval": {"max_depth_eval": 10, "min_depth_eval": 0.001, "garg_crop": False, "eigen_crop": True}}
_NEWCRFS_KITTI = copy.deepcopy(_NEWCRFS_NYU)  # json/kitti/newcrfs/newcrfs_github_eval.json
_NEWCRFS_KITTI["dataset"]["data_type"] = "KITTI"
_NEWCRFS_KITTI["eval"].update(max_depth_eval=80, garg_crop=True, eigen_crop=False)
_ADABINS_NYU = {  # json/nyu/adabins/adabins_cham_per_batch.json (batch 16: BASELINE configs[1])
    "model": {"name": "adabins", "num_bins": 256, "bn_momentum": 0.1},
    "loss": {"alpha": 10.0, "beta": 0.15, "per_image": False, "chamfer_weight": 0.1},
    "dataset": {"data_type": "NYU"}, "dataloader": {"batch_size": 16},
    "optimizer": {"lr": 0.000357, "weight_decay": 0.1},
    "scheduler": {"name": "onecycle", "pct_start": 0.3, "div_factor": 25, "final_div_factor": 100},
    "train": {"epoch": 25, "num_accum": 1, "grad_norm": 0.1},
    "eval": {"max_depth_eval": 10, "min_depth_eval": 0.001, "garg_crop": False, "eigen_crop": True}}
_DFV8_NYU = {  # json/kitti/depthformer/depthformer_v8_cham_loss_per_image_4gpu.json at the NYU crop
    "model": {"name": "depthformer_v8", "hidden_dim": 256, "num_heads": 4, "num_bins": 256, "num_aux": 256,
              "img_size": [480, 640], "bn_momentum": 0.1, "attn_drop_prob": 0.1, "drop_prob": 0.2},
    "loss": {"alpha": 10.0, "beta": 0.5, "per_image": True, "chamfer_weight": 0.1},
    "dataset": {"data_type": "NYU"}, "dataloader": {"batch_size": 8},
    "optimizer": {"lr": 0.00032, "weight_decay": 0.1},
    "scheduler": {"name": "onecycle", "pct_start": 0.15, "div_factor": 25, "final_div_factor": 100},
    "train": {"epoch": 50, "num_accum": 1, "grad_norm": 0.1},
    "eval": {"max_depth_eval": 10, "min_depth_eval": 0.001, "garg_crop": False, "eigen_crop": True}}

_ODA2_KITTI = {  # json/kitti/oda2/oda2_red_order_swin2.json
    "model": {"name": "oda2_red_order_swin2", "encoder_type": "large", "dec_dim": 512, "num_heads": 8,
              "num_repeats": 3, "num_emb": 128, "window_size": 8, "drop_prob": 0.0, "attn_drop_prob": 0.0,
              "bn_momentum": 0.1},
    "loss": {"alpha": 10.0, "beta": 0.15, "per_image": True, "si_weight": 1.0},
    "dataset": {"data_type": "KITTI"}, "dataloader": {"batch_size": 8},
    "optimizer": {"lr": 1e-4, "betas": [0.9, 0.999], "weight_decay": 0.1, "eps": 1e-6, "same_lr": True},
    "scheduler": {"name": "onecycle", "pct_start": 0.25, "div_factor": 25, "final_div_factor": 100,
                  "cycle_momentum": False},
    "train": {"epoch": 24, "num_accum": 2, "grad_norm": 0.1},
    "eval": {"max_depth_eval": 80, "min_depth_eval": 0.001, "garg_crop": True, "eigen_crop": False}}

WORKLOADS = {
    "newcrfs": dict(opt=_NEWCRFS_NYU, model="NewCRFs-L07", h=480, w=640,
                    workload="NewCRFs Swin-L (large07) train step, NYU 480x640",
                    ref_cfg="json/nyu/newcrfs/newcrfs_github_eval.json"),
    "newcrfs_kitti": dict(opt=_NEWCRFS_KITTI, model="NewCRFs-L07", h=352, w=1216,
                          workload="NewCRFs Swin-L (large07) train step, KITTI 352x1216",
                          ref_cfg="json/kitti/newcrfs/newcrfs_github_eval.json"),
    # the reference's real KITTI train crop (dataset/depth_dataset.py:52: random 352x704 crop)
    "newcrfs_kitti704": dict(opt=_NEWCRFS_KITTI, model="NewCRFs-L07", h=352, w=704,
                             workload="NewCRFs Swin-L (large07) train step, KITTI 352x704 (train crop)",
                             ref_cfg="json/kitti/newcrfs/newcrfs_github_eval.json"),
    "adabins": dict(opt=_ADABINS_NYU, model="AdaBins-B5", h=480, w=640,
                    workload="AdaBins EfficientNet-B5 train step, NYU 480x640",
                    ref_cfg="json/nyu/adabins/adabins_cham_per_batch.json"),
    "depthformer": dict(opt=_DFV8_NYU, model="DepthformerV8-B5", h=480, w=640,
                        workload="Depthformer v8 train step, NYU 480x640 (fp32)",
                        ref_cfg="json/kitti/depthformer/depthformer_v8_cham_loss_per_image_4gpu.json"),
    # BASELINE configs[4]: bf16 mixed precision (bf16 GEMM operands, fp32 accumulate / master
    # weights / optimizer) with the whole train step captured in one hipGraph
    "depthformer_bf16": dict(opt=_DFV8_NYU, model="DepthformerV8-B5", h=480, w=640, precision="bf16", graph=True,
                             workload="Depthformer v8 train step, NYU 480x640, bf16 mixed precision, hipGraph",
                             ref_cfg="json/kitti/depthformer/depthformer_v8_cham_loss_per_image_4gpu.json"),
    # SURVEY §8f-4 (not a BASELINE config): ODA2 ordered-swin2, KITTI 352x704 (resized to 448x896
    # inside), batch 8 x num_accum 2 as configured
    "oda2": dict(opt=_ODA2_KITTI, model="ODA2-OrderedSwin2-L", h=352, w=704,
                 workload="ODA2 ordered-swin2 (Swin-L) train step, KITTI 352x704",
                 ref_cfg="json/kitti/oda2/oda2_red_order_swin2.json"),
}
# The default line (BASELINE.json metric, NeW-CRFs NYU) carries every other single-GPU
# BASELINE config as a compact secondary: configs[2] (NeW-CRFs KITTI 352x1216 bs 8),
# configs[1] (AdaBins NYU bs 16) and configs[4] at N GPUs (Depthformer v8 bf16 + hipGraph).
SECONDARIES = {"newcrfs_kitti": 8, "newcrfs_kitti704": 8, "adabins": 16, "depthformer_bf16": 8}
SECONDARY_CPU_BUDGET_S = 8.0  # each secondary's CPU baseline: a shorter sample (the headline's is 20 s)
# HBM bytes per launch of the roofline kernel family, from the committed
# rocprofv3 --pmc passes (tools/pmc_traffic.py; FETCH_SIZE doubled per the
# gfx950 correction).  None when no profile matches the kernel.
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")
KERNEL_NAME = {0: "KCONTIG", 1: "MNCONTIG", 2: "CONV"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="newcrfs", choices=sorted(WORKLOADS))
    ap.add_argument("--config", default=None, help="a reference-format JSON config (overrides --model)")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the secondary workloads")
    ap.add_argument("--secondaries", default=",".join(SECONDARIES),
                    help="comma list of secondary workloads on the default line (subset of " +
                         ",".join(SECONDARIES) + ")")
    ap.add_argument("--precision", default=None, choices=["fp32", "fp32e", "bf16"],
                    help="matmul precision (default: the workload's). fp32: exact-product fp32 MFMA; fp32e: "
                         "fp32 via three exact bf16 planes on the bf16 MFMA (fp32 error); bf16: bf16 operands, "
                         "fp32 accumulate")
    ap.add_argument("--graph", action="store_true", help="capture the whole train step in a hipGraph")
    ap.add_argument("--data", default="synthetic", choices=["synthetic", "synthetic-files"],
                    help="synthetic-files: also time the real-data front end -- NYU-format JPEG/PNG files "
                         "decoded by DepthDataset in DataLoader workers, collate_raw, GpuSampleTransform on "
                         "the GPU -- feeding the same train step (reported beside the synthetic rate)")
    ap.add_argument("--data-workers", type=int, default=4)
    ap.add_argument("--ddp", action="store_true",
                    help="N = 1: run the data-parallel step anyway -- a world-1 RCCL group, GradAllReduce "
                         "buckets and their all-reduces (the N > 1 code path on one GPU)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: launcher/gloo plumbing check only (a toy model, not a measurement)")
    return ap.parse_args()


# --------------------------------------------------------------------------- launcher
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """--gpus N > 1 without a torchrun environment: run N ranks (one per GPU) under
    torch.distributed.run as a child process, before this process touches the GPU, and
    return its exit code."""
    if args.device == "cuda":
        visible = torch.cuda.device_count()  # does not initialise the GPU on this image
        if args.gpus > visible:
            print(f"bench: --gpus {args.gpus} but only {visible} GPU(s) visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def _progress(msg):
    """A line on stderr per bench phase (the GPU harness kills a command silent for 3 min)."""
    print(f"bench[{os.environ.get('RANK', '0')}]: {msg}", file=sys.stderr, flush=True)


# --------------------------------------------------------------------------- data
def synthetic_batch(B, H, W, device, seed, data_type="NYU"):
    """ImageNet-normalised uniform images; NYU depth U(0.5, 10) inside the
    [45:472, 43:608] valid region, KITTI depth U(1, 80) at a Bernoulli(0.15) LiDAR-like mask."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    img = torch.rand(B, 3, H, W, generator=g)
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    img = (img - mean) / std  # depth_dataset.py:290 (ImageNet Normalize)
    if data_type == "NYU":
        gt = torch.rand(B, 1, H, W, generator=g) * 9.5 + 0.5
        valid = torch.zeros(B, 1, H, W)
        valid[:, :, 45 * H // 480:472 * H // 480, 43 * W // 640:608 * W // 640] = 1  # NYU valid region
    else:
        gt = torch.rand(B, 1, H, W, generator=g) * 79.0 + 1.0
        valid = (torch.rand(B, 1, H, W, generator=g) < 0.15).float()
    return img.to(device), (gt * valid).to(device)


# --------------------------------------------------------------------------- real-data front end
class FilePipeline:
    """SURVEY §8f-2 / dataset/depth_dataset.py:166-284 on files: `n_files` synthetic NYU-format
    frames written once to a temporary directory (RGB JPEG, quality 95, and a 16-bit PNG depth
    in millimetres, saving_factor 1000 -- the reference's NYU layout), then per step
    DepthDataset.__getitem__ (Pillow decode) in `workers` DataLoader worker processes,
    collate_raw into pinned host batches, and GpuSampleTransform (rotate, crop, flip, colour
    augmentation, normalisation: one libmdemi sweep) on the GPU.  The workers are forked here,
    before this process touches the GPU, and only decode."""

    def __init__(self, B, H, W, data_type, n_files, workers, seed=0):
        import tempfile

        import numpy as np
        from PIL import Image
        from mdemi.dataset import DepthDataset, collate_raw
        if data_type != "NYU":
            raise SystemExit("bench: --data synthetic-files writes NYU-format frames (the default workload)")
        self.tmp = tempfile.TemporaryDirectory(prefix="mdemi_bench_files_")
        rng = np.random.default_rng(seed)
        yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
        names = []
        for i in range(n_files):  # smooth colour fields + noise (JPEG sizes like photographs') and a depth ramp
            ph = rng.uniform(0, 6.28, 3)
            rgb = np.stack([127 + 80 * np.sin(xx / (37 + 11 * c) + yy / (53 - 7 * c) + ph[c]) for c in range(3)], -1)
            rgb = np.clip(rgb + rng.normal(0, 12, rgb.shape), 0, 255).astype(np.uint8)
            dep = (1000 * (0.5 + 9.0 * (xx / W) * (0.6 + 0.4 * np.sin(yy / 41 + ph[0])) ** 2)).astype(np.uint16)
            Image.fromarray(rgb).save(os.path.join(self.tmp.name, f"rgb_{i:04d}.jpg"), quality=95)
            Image.fromarray(dep).save(os.path.join(self.tmp.name, f"sync_depth_{i:04d}.png"))
            names.append(f"/rgb_{i:04d}.jpg /sync_depth_{i:04d}.png 518.8579\n")
        self.bytes_on_disk = sum(os.path.getsize(os.path.join(self.tmp.name, f)) for f in os.listdir(self.tmp.name))
        self.ds = DepthDataset(self.tmp.name, "NYU", "train", img_size=(H, W), filenames=names)
        sampler = torch.utils.data.RandomSampler(self.ds, replacement=True, num_samples=1 << 30,
                                                 generator=torch.Generator().manual_seed(seed))
        self.loader = torch.utils.data.DataLoader(self.ds, batch_size=B, sampler=sampler, num_workers=workers,
                                                  collate_fn=collate_raw, pin_memory=True, drop_last=True,
                                                  persistent_workers=workers > 0, prefetch_factor=4 if workers else None,
                                                  multiprocessing_context="fork" if workers else None)
        self.it = iter(self.loader)  # forks the workers now (before any HIP call in this process)
        self.n_files, self.workers = n_files, workers
        self.tf = None

    def next(self):
        import random as _random
        if self.tf is None:
            self.tf = self.ds.transform()
            self.rnd = _random.Random(0)
        b = next(self.it)
        img, gt, _ = self.tf(b["image"], b["depth"], rnd=self.rnd)
        return img, gt

    def close(self):
        del self.it
        self.tmp.cleanup()


def measure_files(args, trainer, pipe, B, world):
    """The train step fed from the file pipeline: W warm-up steps, then K timed steps
    (barrier + synchronize on both sides, as in measure), each = next decoded batch ->
    GpuSampleTransform -> Trainer.step.  Also the front end alone over K batches."""
    na = trainer.num_accum
    for _ in range(max(args.warmup, 1)):
        trainer.step([pipe.next() for _ in range(na)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step([pipe.next() for _ in range(na)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    # front end alone: decode (workers) + pinned H2D + augment sweep, over more batches than the
    # workers hold prefetched (workers x prefetch_factor), so the rate is the decode rate
    nfe = max(args.steps, 6 * max(pipe.workers, 1) * 4)
    t0 = time.perf_counter()
    for _ in range(nfe):
        pipe.next()
    torch.cuda.synchronize()
    fe = (time.perf_counter() - t0) * args.steps / nfe
    return {"images_per_sec": round(B * na * world * args.steps / elapsed, 3),
            "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "front_end_alone_images_per_sec": round(B * na * args.steps / fe, 2),
            "workers": pipe.workers, "files": pipe.n_files, "bytes_on_disk": pipe.bytes_on_disk,
            "pipeline": "DepthDataset.__getitem__ (Pillow JPEG/PNG decode, DataLoader workers) -> collate_raw "
                        "(pinned) -> GpuSampleTransform (mdemi_augment: rotate/crop/flip/colour/normalise) -> "
                        "Trainer.step"}


# --------------------------------------------------------------------------- roofline
def _gemm_alg_bytes(A, B, M, N, K, kw, ob=4.0):
    """Algorithmic HBM bytes of one GEMM launch: every operand read once (ob bytes per element:
    4 fp32, 2 on the bf16-operand path), C written once in fp32 (plus its bf16 copy when one is
    requested); conv operands count the NHWC activation, not its im2col."""
    def operand(layout, rows, cols):
        if layout == 2:  # implicit im2col: the activation tensor
            g = kw["conv"]
            return ob * g.n * g.h * g.w * g.c
        return ob * rows * cols
    batch = kw.get("batch", 1)
    b = operand(kw.get("a_layout"), M, K) + operand(kw.get("b_layout"), K, N)
    b *= batch if kw.get("a_layout") != 2 else 1
    c = 4.0 * M * N * batch
    b += c * (2 if kw.get("beta", 0.0) else 1)
    if kw.get("c16") is not None:
        b += c / 2
    for extra in ("aux", "residual", "preact"):
        if kw.get(extra) is not None:
            b += c
    return b


class _HbmTimers:
    """HIP events around the C entry points of the memory-heavy fused ops during the
    instrumented step (the events bracket the entry's own launches on its stream, so no
    host-side gap between kernels is counted), with their algorithmic bytes -> achieved GB/s
    against the 8 TB/s HBM peak:
      binhead_nhwc_fwd/bwd (SURVEY §8d's HBM-bound row): fwd reads the logits and writes
        pred + the (max, sum) row stats, 4*B*HW*(K+3) B; bwd reads logits, pred, stats and
        dpred and writes dlogits, 4*B*HW*(2K+4) B;
      winattn_fwd/bwd (fused shifted-window attention): fwd reads q, k, v and
        writes out, 16*C B per token; bwd reads q, k, v, out, dout and writes dq, dk, dv,
        32*C B per token (the window's MFMA work rides on the same pass).  The forward entry
        also launches the small relative-position-bias expansion, which the backward reuses;
        the backward adds the bias gradient's column sum and scatter: a few us each, counted in
        the window."""

    def __init__(self, lib):
        def wa_bytes(per_token):
            def f(args):
                d = args[0]._obj  # ctypes.byref(WinAttnDesc)
                return per_token * d.heads * d.head_dim * d.B * d.H * d.W
            return f

        def wa_mfma(n_mfma):  # v_mfma_f32_32x32x2_f32 issued per (window, head): 4096 FLOP each
            def f(args):
                d = args[0]._obj
                nwin = d.B * -(-d.H // d.window) * -(-d.W // d.window)
                return 4096.0 * n_mfma * nwin * d.heads
            return f

        self.specs = {"mdemi_binhead_nhwc_fwd": ("binhead_nhwc_fwd", lambda a: 4.0 * a[4] * a[5] * (a[6] + 3)),
                      "mdemi_binhead_nhwc_bwd": ("binhead_nhwc_bwd", lambda a: 4.0 * a[7] * a[8] * (2 * a[9] + 4)),
                      "mdemi_winattn_fwd": ("winattn_fwd", wa_bytes(16.0)),
                      "mdemi_winattn_bwd_bias": ("winattn_bwd", wa_bytes(32.0))}
        # window attention is bound by its fp32 MFMA work, not by bytes: 49 tokens padded to 64,
        # 120 (forward) / 284 (backward) v_mfma_f32_32x32x2_f32 per (window, head) in the
        # kernels' instruction streams (winattn.hip; counted from the gfx950 ISA)
        self.mfma = {"winattn_fwd": wa_mfma(120), "winattn_bwd": wa_mfma(284)}
        self.lib = lib
        self.orig = {entry: getattr(lib, entry) for entry in self.specs}
        self.recs = {name: [] for name, _ in self.specs.values()}
        for entry, (name, nbytes) in self.specs.items():
            setattr(lib, entry, self._wrap(self.orig[entry], nbytes, self.mfma.get(name), self.recs[name]))

    @staticmethod
    def _wrap(fn, nbytes, nflops, recs):
        def timed(*args):
            _spin()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(torch.cuda.current_stream())
            rc = fn(*args)
            e.record(torch.cuda.current_stream())
            recs.append((nbytes(args), nflops(args) if nflops else 0.0, s, e))
            return rc
        return timed

    def restore(self):
        for entry, fn in self.orig.items():
            setattr(self.lib, entry, fn)

    def summary(self):
        out = {}
        for name, recs in self.recs.items():
            if not recs:
                continue
            t = sum(s.elapsed_time(e) for _, _, s, e in recs) * 1e-3
            by = sum(b for b, _, _, _ in recs)
            fl = sum(f for _, f, _, _ in recs)
            out[name] = {"launches": len(recs), "avg_us": round(t / len(recs) * 1e6, 1),
                         "algorithmic_bytes_per_launch": round(by / len(recs)),
                         "achieved_GBps": round(by / t / 1e9, 1),
                         "frac_of_hbm_peak": round(by / t / 1e9 / HBM_PEAK_GBS, 4)}
            if fl:
                out[name].update({"bound": "mfma", "mfma_flops_per_launch": round(fl / len(recs)),
                                  "mfma_tflops": round(fl / t / 1e12, 2),
                                  "frac_of_fp32_mfma_peak": round(fl / t / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)})
        return out or None


GEMM_ENTRIES = ("mdemi_gemm_f32", "mdemi_gemm_bf16", "mdemi_gemm_f32e", "mdemi_gemm_bf16x")
SPIN_CYCLES = 60000  # ~25 us of torch.cuda._sleep ahead of each timed launch


def _spin():
    """Keep the GPU busy while the host enqueues [start event, kernel(s), end event], so the
    events bracket device time only -- not the host's launch latency of an eager step, which on
    the configs[4] step's 20-40 us GEMMs is as long as the kernels (round 6: 66 us by events
    around the Python call vs 37 us in the rocprofv3 trace)."""
    sleep = getattr(torch.cuda, "_sleep", None)
    if sleep is not None:
        sleep(SPIN_CYCLES)


def gemm_roofline(trainer, batches):
    """One instrumented (eager, even for a captured trainer) step: HIP events around every
    libmdemi GEMM entry-point call on its stream (the GEMM kernel and, for split K, its slab
    reduce; not the bf16 casts or bias column sums gemm() may launch first), each preceded by a
    spin kernel so the events time the device only; algorithmic FLOPs (2*M*N*K per GEMM) and
    bytes / measured kernel time, per kernel family."""
    from mdemi import functional as mf
    from mdemi import _lib as L
    lib = L.load()
    recs, pending = [], []
    orig = mf.gemm
    orig_c = {n: getattr(lib, n) for n in GEMM_ENTRIES}

    def wrap_c(fn):
        def f(*args):
            _spin()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(torch.cuda.current_stream())
            rc = fn(*args)
            e.record(torch.cuda.current_stream())
            if pending and pending[-1] is None:
                pending[-1] = (s, e)
            return rc
        return f

    def timed(A, B, C, M, N, K, **kw):
        pending.append(None)
        try:
            out = orig(A, B, C, M, N, K, **kw)
        finally:
            ev = pending.pop()
        if ev is None:
            return out
        path = mf.LAST_GEMM[0]  # "b16": bf16 operands in HBM (gemm_b16_kernel)
        key = (path, kw.get("a_layout"), kw.get("b_layout"), kw.get("a_op", 0), kw.get("b_op", 0))
        recs.append((key, 2.0 * M * N * K * kw.get("batch", 1),
                     _gemm_alg_bytes(A, B, M, N, K, kw, ob=2.0 if path == "b16" else 4.0), ev[0], ev[1]))
        return out

    mf.gemm = timed
    for n, fn in orig_c.items():
        setattr(lib, n, wrap_c(fn))
    hbm = _HbmTimers(lib)
    try:
        with mf.matmul_precision(trainer.precision):
            trainer._eager_step(batches)
        torch.cuda.synchronize()
    finally:
        mf.gemm = orig
        for n, fn in orig_c.items():
            setattr(lib, n, fn)
        hbm.restore()
    trainer._hbm_kernels = hbm.summary()
    by = {}
    for key, fl, by_alg, s, e in recs:
        t = s.elapsed_time(e) * 1e-3
        a = by.setdefault(key, [0.0, 0.0, 0, 0.0])
        a[0] += fl
        a[1] += t
        a[2] += 1
        a[3] += by_alg
    tot_fl = sum(v[0] for v in by.values())
    tot_t = sum(v[1] for v in by.values())
    dom = max(by.items(), key=lambda kv: kv[1][1])
    return by, dom, tot_fl, tot_t


def profiled_traffic(regex, workload):
    try:
        with open(TRAFFIC_FILE) as f:
            prof = json.load(f)
    except (OSError, ValueError):
        return None
    fam = prof.get(workload, {}).get("families", {}).get(regex)
    return None if fam is None else fam.get("traffic_bytes_per_launch")


def _family(key, prec):
    """(kernel name, MFMA peak TF/s, rocprofv3 regex) of a GEMM family key (path, al, bl, aop, bop)."""
    path, al, bl, aop, bop = key
    if path == "b16":  # bf16 operands in HBM, direct-to-LDS (gemm_b16_kernel.h)
        return "gemm_b16_kernel", BF16_MFMA_PEAK_TFLOPS, f"gemm_b16_kernel<{al}, {bl},"
    if prec == "fp32":  # register-staged gemm_f32_kernel and direct-to-LDS gemm_glds_kernel: one family
        return "gemm_f32_kernel|gemm_glds_kernel", FP32_MFMA_PEAK_TFLOPS, f"gemm_f32<{al}, {bl}, {aop}, {bop}>"
    np_ = 1 if prec == "bf16" else 3  # the 16-bit family: NP = 1 (bf16) or 3 (fp32e) planes
    return ("gemm_m16_kernel", BF16_MFMA_PEAK_TFLOPS if prec == "bf16" else F32E_MFMA_PEAK_TFLOPS,
            f"gemm_m16_kernel<{al}, {bl}, {aop}, {bop}, {np_},")


def _bound(fl, t, alg, peak):
    """The roofline that bounds a family: MFMA when its algorithmic intensity (FLOP per HBM
    byte) exceeds the machine balance peak / 8 TB/s, else HBM."""
    if fl / max(alg, 1.0) >= peak * 1e12 / (HBM_PEAK_GBS * 1e9):
        return "mfma", fl / t / 1e12, peak, "TFLOP/s"
    return "hbm", alg / t / 1e9, HBM_PEAK_GBS, "GB/s"


def roofline_entry(trainer, batches, workload_key, ms):
    by, dom, tot_fl, tot_t = gemm_roofline(trainer, batches)
    key, (fl, t, cnt, alg) = dom
    _, al, bl, aop, bop = key
    prec = trainer.precision
    kname, peak, regex = _family(key, prec)
    bound, ach, roof_peak, unit = _bound(fl, t, alg, peak)
    traffic = profiled_traffic(regex, workload_key)
    alg_pl = alg / cnt
    roof = {"bound": bound, "achieved": round(ach, 2), "peak": roof_peak, "unit": unit,
            "frac": round(ach / roof_peak, 4),
            "traffic": traffic, "traffic_unit": "HBM bytes/launch (rocprofv3 PMC)",
            "algorithmic_bytes": round(alg_pl), "traffic_over_algorithmic":
                (round(traffic / alg_pl, 3) if traffic else None),
            "kernel": f"{kname}<{KERNEL_NAME[al]},{KERNEL_NAME[bl]},{aop},{bop}> ({prec}; all pipelining variants)",
            "kernel_regex": regex, "launches": cnt, "avg_launch_us": round(t / cnt * 1e6, 2),
            "flops_per_launch": fl / cnt, "tflops": round(fl / t / 1e12, 2)}
    fams = {}
    for k, v in sorted(by.items(), key=lambda kv: -kv[1][1]):
        b, a, pk, u = _bound(v[0], v[1], v[3], _family(k, prec)[1])
        fams[f"{k[0]}:{KERNEL_NAME[k[1]]},{KERNEL_NAME[k[2]]},{k[3]},{k[4]}"] = {
            "launches": v[2], "ms_per_step": round(v[1] * 1e3, 3), "tflops": round(v[0] / v[1] / 1e12, 2),
            "algorithmic_GBps": round(v[3] / v[1] / 1e9, 1), "bound": b, "frac": round(a / pk, 4)}
    extra = {"gemm_all": {"achieved_tflops": round(tot_fl / tot_t / 1e12, 2), "gemm_ms_per_step": round(tot_t * 1e3, 2),
                          "gemm_tflop_per_step": round(tot_fl / 1e12, 3),
                          "frac": round(tot_fl / tot_t / 1e12 / peak, 4), "families": fams},
             "step_mfma_frac": round(tot_fl / (ms * 1e-3) / 1e12 / peak, 4)}
    return roof, extra


# --------------------------------------------------------------------------- CPU baseline
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _usable_cpus():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(model, opt, H, W, budget_s, all_cores=True):
    """The oracle (CPU restatement of the reference path: oracle/newcrfs.py, oracle/adabins.py,
    oracle/depthformer.py) timed on the host cores: fp32 forward + loss + backward + clipped
    AdamW step at batch 1 with the same weights, 2 warm-up steps, then as many timed steps
    (1-5) as fit the budget."""
    from oracle import metrics as omet
    name = opt["model"]["name"]
    lo = opt["loss"]
    dmin, dmax = opt["eval"]["min_depth_eval"], opt["eval"]["max_depth_eval"]
    threads = min(CPU_SHARE_PER_GPU, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    P = {k: v.detach().float().cpu().clone().requires_grad_(torch.is_floating_point(v))
         for k, v in model.state_dict().items()}
    params = [v for v in P.values() if v.requires_grad]
    copt = torch.optim.AdamW(params, lr=opt["optimizer"]["lr"], weight_decay=opt["optimizer"]["weight_decay"])
    img, gt = synthetic_batch(1, H, W, "cpu", seed=1, data_type=opt["dataset"]["data_type"])
    if name == "adabins":
        from oracle import adabins as oab
        fwd = lambda: oab.unet_adaptive_bins(P, img, dmin, dmax)  # noqa: E731
    elif name == "depthformer_v8":
        from oracle import depthformer as odf
        opt_m = dict(opt["model"], attn_drop_prob=0.0, drop_prob=0.0)
        fwd = lambda: odf.depthformer_v8_full(P, img, opt_m, dmin, dmax)  # noqa: E731
    elif name == "oda2_red_order_swin2":
        from oracle import oda2 as oo
        m = opt["model"]
        enc = {"depths": (2, 2, 18, 2), "num_heads": (6, 12, 24, 48) if m["encoder_type"] in ("large", "L")
               else (4, 8, 16, 32)}
        dec = {k: m[k] for k in ("num_heads", "num_repeats", "num_emb")}
        dec.update(window_size=m.get("window_size", 8), neck_type=m.get("neck_type", "red"),
                   output_scale=m.get("output_scale", 4), bias_type=m.get("bias_type", "depth"))
        fwd = lambda: oo.oda2_model(P, img, enc, dec, dmax)[:2]  # noqa: E731  (out, outs)
    else:
        from oracle import newcrfs as onc
        fwd = lambda: onc.newcrf_depth(P, img, "large07", max_depth=dmax)  # noqa: E731
    cham = float(lo.get("chamfer_weight", 0.0))

    def up(p):
        if p.shape[-2:] != gt.shape[-2:]:
            p = torch.nn.functional.interpolate(p, gt.shape[-2:], mode="bilinear", align_corners=True)
        return p

    def step():
        out = fwd()
        if name == "oda2_red_order_swin2":  # SILog over every output (train/builder.py TrainLoss)
            outs = out[1]
            loss = sum(omet.silog_loss(up(o), gt, dmin, lo["alpha"], lo["beta"], lo["per_image"]) for o in outs)
            loss = loss * (float(lo.get("si_weight", 1.0)) / len(outs))
        else:
            pred = up(out[0] if isinstance(out, tuple) else out)
            loss = omet.silog_loss(pred, gt, dmin, lo["alpha"], lo["beta"], lo["per_image"])
        if cham > 0:
            from oracle.adabins import bins_chamfer_loss
            loss = loss + cham * bins_chamfer_loss(out[1], gt, dmin, from_edges=(name == "adabins"))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, opt["train"]["grad_norm"])
        copt.step()
        copt.zero_grad(set_to_none=True)

    def timed(threads, budget):
        torch.set_num_threads(threads)
        t0 = time.perf_counter()
        step()
        step()  # 2 warm-up steps
        per = (time.perf_counter() - t0) / 2
        n = max(1, min(5, int(budget / max(per, 1e-3))))
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        return (time.perf_counter() - t0) / n, n

    dt, n = timed(threads, budget_s)
    res = {"value": round(1.0 / dt, 4), "unit": "images/sec", "cores": threads, "kind": "port",
           "sample": f"oracle {name} fp32 train step (fwd+SILog{'+chamfer' if cham else ''}+bwd+clip+AdamW), "
                     f"batch 1 at {H}x{W}, {n} timed steps after 2 warm-up, {threads} threads (the box's "
                     f"per-GPU CPU share), {os.cpu_count()} host CPUs visible, CPU: {_cpu_model()}"}
    # SURVEY §8d asks for every physical core: the same sample on all the CPUs this process may
    # actually use (affinity, capped by the cgroup CPU quota -- oversubscribing a quota only
    # slows the sample down), reported beside the share when that is more
    allc = _usable_cpus()
    _progress(f"cpu_baseline: {threads} threads {1.0 / dt:.3f} img/s; usable CPUs {allc}")
    res["usable_cpus"] = allc
    if all_cores and allc > threads and budget_s > 0:
        dt2, n2 = timed(allc, budget_s / 2)
        res["all_cores"] = {"value": round(1.0 / dt2, 4), "cores": allc, "timed_steps": n2}
    torch.set_num_threads(threads)
    return res


# --------------------------------------------------------------------------- one measurement
def measure(args, opt, key, H, W, B, rank, world, device, with_roofline, precision="fp32", graph=False):
    """Build the trainer from `opt`, run W warm-up + K timed steps; returns a dict."""
    from mdemi.train import build_from_config
    opt = copy.deepcopy(opt)
    opt["dataloader"]["batch_size"] = B
    torch.cuda.synchronize(device)  # initialises the device context the peak counter needs
    torch.cuda.reset_peak_memory_stats(device)
    torch.manual_seed(0)
    trainer = build_from_config(opt, device=device, world=world, precision=precision, graph=graph,
                                ddp=(True if getattr(args, "ddp", False) else None))
    na = trainer.num_accum
    batches = [synthetic_batch(B, H, W, device, seed=1000 + 7 * rank + i, data_type=opt["dataset"]["data_type"])
               for i in range(na)]
    _progress(f"{key}: built (B={B} {H}x{W} {precision}{' graph' if graph else ''}), warm-up")
    for _ in range(args.warmup):
        trainer.step(batches)
    torch.cuda.synchronize()
    _progress(f"{key}: timing {args.steps} steps")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step(batches)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    res = {"elapsed": elapsed, "ms": elapsed / args.steps * 1e3, "images": B * na * world * args.steps,
           "loss": float(loss.item()), "num_accum": na, "trainer": trainer,
           # peak device memory of the build + warm-up + timed steps (bf16 storage: incl. the copies)
           "peak_mem_GB": round(torch.cuda.max_memory_allocated(device) / 1e9, 2)}
    if trainer.ddp is not None:  # isolated cost of the whole gradient exchange (no overlap): an upper bound on exposed comm
        ddp = trainer.ddp
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(3):
            ddp.allreduce_all()
        torch.cuda.synchronize()
        iso = (time.perf_counter() - t0) / 3 * 1e3
        res["allreduce"] = {"grad_bytes": sum(ddp.bucket_bytes), "buckets": len(ddp.buckets),
                            "isolated_ms": round(iso, 2), "share_of_step_upper_bound": round(iso / res["ms"], 4),
                            "bus_GBps": (round(2 * (world - 1) / world * sum(ddp.bucket_bytes) / (iso * 1e-3) / 1e9, 1)
                                         if world > 1 else None),
                            "last_launch_order": ddp.last_launch_order}
        res["allreduce"]["overlap"] = ddp_overlap(trainer, batches)
    _progress(f"{key}: {res['ms']:.1f} ms/step")
    if with_roofline:
        res["roofline"], res["extra"] = roofline_entry(trainer, batches, key, res["ms"])
        if getattr(trainer, "_hbm_kernels", None):
            res["extra"]["hbm_kernels"] = trainer._hbm_kernels
    return res


XGMI_RING_BUS_GBPS = 300.0  # assumed RCCL ring bus bandwidth over xGMI at 8 GPUs


def ddp_overlap(trainer, batches, n_model=8, bus_gbps=XGMI_RING_BUS_GBPS):
    """One traced eager step (GradAllReduce.trace_events): for every bucket, when it became
    ready and when it was launched (strict index order), in ms before the end of backward, from
    HIP events on the compute stream.  From those offsets, the exposed communication an
    n_model-GPU ring would leave: bucket i's all-reduce takes 2 (n-1)/n bytes_i / bus on the one
    communication stream, starting at max(its launch, the previous bucket's end); whatever runs
    past the end of backward is exposed."""
    from mdemi import functional as mf
    ddp = trainer.ddp
    ddp.trace_events = True
    ddp.reset()
    try:
        with mf.matmul_precision(trainer.precision):
            trainer._eager_step(batches)
        torch.cuda.synchronize()
        tr = ddp.trace_offsets()
    finally:
        ddp.trace_events = False
        ddp.reset()
    if tr is None:
        return None
    t_free, exposed_by = None, []
    for row in tr["buckets"]:  # times relative to the end of backward (negative = before it)
        start = -row["launch_before_end_ms"]
        if t_free is not None:
            start = max(start, t_free)
        dur = 2.0 * (n_model - 1) / n_model * row["bytes"] / (bus_gbps * 1e9) * 1e3
        t_free = start + dur
        row["model_ring_ms"] = round(dur, 3)
        row["model_done_after_end_ms"] = round(t_free, 3)
    exposed = max(0.0, t_free)
    late = [r["bucket"] for r in tr["buckets"] if r["launch_before_end_ms"] < r["ready_before_end_ms"] - 0.05]
    return {"buckets": tr["buckets"], "ready_order": tr["ready_order"],
            "ready_order_is_index_order": tr["ready_order"] == sorted(tr["ready_order"]),
            "held_back_buckets": late,
            "model": f"{n_model}-GPU ring all-reduce at {bus_gbps:g} GB/s bus, buckets serialised on one "
                     "communication stream from their measured launch times",
            "model_exposed_ms": round(exposed, 3)}


def measure_secondary(args, sk, rank, world, device):
    """One secondary BASELINE workload: fewer timed steps than the headline (each is a
    whole-model train step, so 5 steps already average over every kernel), its own
    instrumented roofline step and HBM-kernel rates."""
    wk = WORKLOADS[sk]
    B = SECONDARIES[sk]
    prec = wk.get("precision", "fp32")
    graph = wk.get("graph", False)
    sub = argparse.Namespace(**vars(args))
    sub.steps = max(3, min(args.steps, 5))
    sub.warmup = max(3 if graph else 1, min(args.warmup, 3))  # a captured step: 2 eager + the capture
    sec = measure(sub, wk["opt"], sk, wk["h"], wk["w"], B, rank, world, device, with_roofline=not args.no_roofline,
                  precision=prec, graph=graph)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(sec["trainer"].model, wk["opt"], wk["h"], wk["w"], SECONDARY_CPU_BUDGET_S, all_cores=False)
        if prec != "fp32":
            cpu["sample"] += " (fp32: the CPU path has no bf16 GEMM; the GPU line is bf16)"
    del sec["trainer"]
    out = {"workload": wk["workload"], "reference_config": wk["ref_cfg"], "per_gpu_batch": B,
           "image": [wk["h"], wk["w"]], "matmul_precision": prec, "hipgraph": graph, "steps": sub.steps,
           "images_per_sec": round(sec["images"] / sec["elapsed"], 3), "ms_per_step": round(sec["ms"], 2),
           "loss": round(sec["loss"], 5), "peak_mem_GB": sec["peak_mem_GB"], "cpu_baseline": cpu}
    if "roofline" in sec:
        out["roofline"] = sec["roofline"]
        out["step_mfma_frac"] = sec["extra"]["step_mfma_frac"]
        out["gemm_all_frac"] = sec["extra"]["gemm_all"]["frac"]
        if "hbm_kernels" in sec["extra"]:
            out["hbm_kernels"] = sec["extra"]["hbm_kernels"]
        if sk == "newcrfs_kitti":  # 2404.7 GFLOP per image per train step at 352x1216
            out["survey_flop_frac"] = round(2404.7e9 * sec["images"] / sec["elapsed"] / world / 1e12 /
                                            FP32_MFMA_PEAK_TFLOPS, 4)
    if "allreduce" in sec:
        out["allreduce"] = sec["allreduce"]
    return out


def measure_configs0(args, device, budget_s):
    """BASELINE configs[0]: AdaBins EfficientNet-B5 forward on one 640x480 NYU crop.  The
    reference states it as a PyTorch-CPU plumbing case; here the oracle's fp32 forward (the CPU
    restatement, oracle/adabins.py) is timed on the host cores beside the libmdemi eval forward
    of the same weights on the GPU (batch 1, no autograd)."""
    from mdemi.train.builder import build_model
    from oracle import adabins as oab
    opt = copy.deepcopy(_ADABINS_NYU)
    dmin, dmax = opt["eval"]["min_depth_eval"], opt["eval"]["max_depth_eval"]
    torch.manual_seed(0)
    model = build_model(opt).to(device).eval()
    img, _ = synthetic_batch(1, 480, 640, device, seed=1)
    with torch.no_grad():
        for _ in range(3):
            model(img)
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            model(img)
        torch.cuda.synchronize()
        gpu_dt = (time.perf_counter() - t0) / n
    threads = min(CPU_SHARE_PER_GPU, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    P = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    cimg = img.cpu()
    with torch.no_grad():
        t0 = time.perf_counter()
        oab.unet_adaptive_bins(P, cimg, dmin, dmax)  # warm-up
        per = time.perf_counter() - t0
        k = max(1, min(5, int(budget_s / max(per, 1e-3))))
        t0 = time.perf_counter()
        for _ in range(k):
            oab.unet_adaptive_bins(P, cimg, dmin, dmax)
        cpu_dt = (time.perf_counter() - t0) / k
    _progress(f"configs[0]: GPU forward {gpu_dt * 1e3:.2f} ms, CPU oracle forward {cpu_dt * 1e3:.0f} ms")
    return {"workload": "AdaBins EfficientNet-B5 forward (eval), one NYU 480x640 crop (BASELINE configs[0])",
            "reference_config": "json/nyu/adabins/adabins_cham_per_batch.json",
            "gpu_images_per_sec": round(1.0 / gpu_dt, 2), "gpu_ms_per_image": round(gpu_dt * 1e3, 3),
            "cpu_baseline": {"value": round(1.0 / cpu_dt, 4), "unit": "images/sec", "cores": threads, "kind": "port",
                             "sample": f"oracle adabins fp32 forward, batch 1 at 480x640, {k} timed after 1 warm-up, "
                                       f"{threads} threads, CPU: {_cpu_model()}"}}


# --------------------------------------------------------------------------- plumbing (CPU)
def plumbing_main(args, rank, world):
    """--device cpu: the launcher / gloo / barrier / max-over-ranks / JSON path with a toy
    model (no libmdemi); for the CPU tests of the N > 1 launch only."""
    from mdemi.train.ddp import GradAllReduce, broadcast_parameters
    if world > 1:
        dist.init_process_group("gloo")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 1))
    ddp = None
    if world > 1:
        broadcast_parameters(model)
        ddp = GradAllReduce(model, bucket_mb=0.0002)
    optim = torch.optim.AdamW(model.parameters(), lr=1e-3)
    x = torch.randn(8, 32, generator=torch.Generator().manual_seed(rank))

    def step():
        loss = model(x).square().mean()
        loss.backward()
        if ddp is not None:
            ddp.finish()
        optim.step()
        if ddp is not None:
            ddp.zero_grad()
        else:
            optim.zero_grad()
        return loss

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        with torch.no_grad():
            psum = torch.stack([p.detach().double().sum() for p in model.parameters()]).sum()
        lo_hi = torch.stack([-psum, psum])
        dist.all_reduce(lo_hi, op=dist.ReduceOp.MAX)
        identical = bool(-lo_hi[0] == lo_hi[1])
    if rank == 0:
        print(json.dumps({"metric": "plumbing (CPU toy model; not a measurement)", "value": 8 * world * args.steps /
                          elapsed, "unit": "samples/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                          "data": "plumbing", "config": {"workload": "plumbing", "parallelism": f"dp{world}"},
                          "buckets": len(ddp.buckets) if ddp else 0,
                          "launch_order": ddp.last_launch_order if ddp else [],
                          "replicas_identical": identical if world > 1 else True}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# --------------------------------------------------------------------------- main
def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.device == "cpu":
        return plumbing_main(args, rank, world)
    pipe = None
    if args.data == "synthetic-files":  # before any GPU call: the decode workers fork here
        wl0 = WORKLOADS[args.model] if not args.config else None
        if wl0 is None:
            raise SystemExit("bench: --data synthetic-files runs the --model workloads")
        B0 = args.batch or int(wl0["opt"]["dataloader"]["batch_size"])
        pipe = FilePipeline(B0, args.height or wl0["h"], args.width or wl0["w"], wl0["opt"]["dataset"]["data_type"],
                            n_files=max(4 * B0, 32), workers=args.data_workers, seed=rank)
        _progress(f"file pipeline: {pipe.n_files} frames written, {pipe.workers} decode workers")
    if local >= torch.cuda.device_count():
        print(f"bench: local rank {local} has no GPU ({torch.cuda.device_count()} visible)", file=sys.stderr)
        sys.exit(2)
    if world > 1 or args.ddp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if world == 1 and "MASTER_PORT" not in os.environ:  # --ddp without a launcher: a world-1 group
            os.environ.update(MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
    device = torch.device("cuda", local)

    if args.config:
        with open(args.config) as f:
            opt = json.load(f)
        key, ref_cfg = "config", args.config
        img = opt.get("dataset", {}).get("img_size")
        dt = opt.get("dataset", {}).get("data_type", "NYU")
        H, W = (args.height or (img[0] if img else (480 if dt == "NYU" else 352)),
                args.width or (img[1] if img else (640 if dt == "NYU" else 704)))
        wl = dict(model=opt["model"]["name"], workload=f"{opt['model']['name']} train step from {args.config}")
    else:
        key = args.model
        wl = WORKLOADS[key]
        opt, ref_cfg = wl["opt"], wl["ref_cfg"]
        H, W = args.height or wl["h"], args.width or wl["w"]
    B = args.batch or int(opt["dataloader"]["batch_size"])
    precision = args.precision or wl.get("precision", "fp32")
    graph = args.graph or wl.get("graph", False)  # data parallel too: the RCCL all-reduces are in the graph

    res = measure(args, opt, key, H, W, B, rank, world, device, with_roofline=not args.no_roofline,
                  precision=precision, graph=graph)
    value = res["images"] / res["elapsed"]
    files = None
    if pipe is not None:
        _progress("file pipeline: timing")
        files = measure_files(args, res["trainer"], pipe, B, world)
        files["vs_synthetic"] = round(files["images_per_sec"] / value, 4)
        pipe.close()
        _progress(f"file pipeline: {files['images_per_sec']} img/s ({files['vs_synthetic']} of synthetic)")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(res["trainer"].model, opt, H, W, args.cpu_budget_s)
    del res["trainer"]
    torch.cuda.empty_cache()

    secondary = None
    if key == "newcrfs" and not args.no_secondary and args.batch is None and args.height is None:
        secondary = {}
        for sk in [k for k in args.secondaries.split(",") if k]:
            if sk not in SECONDARIES:
                raise SystemExit(f"bench: unknown secondary {sk!r}")
            secondary[sk] = measure_secondary(args, sk, rank, world, device)
            torch.cuda.empty_cache()
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            secondary["configs0_adabins_forward"] = measure_configs0(args, device, SECONDARY_CPU_BUDGET_S)
            torch.cuda.empty_cache()

    if rank == 0:
        line = {
            "metric": ("images/sec (train step) NYU 640x480 bs=8/GPU" if key == "newcrfs" else
                       f"images/sec (train step) {wl['model']} {W}x{H} bs={B}/GPU"),
            "value": round(value, 3), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(res["ms"], 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16" if precision == "bf16" else "fp32",
            "data": "synthetic (random-init weights)",
            "config": {"workload": wl["workload"], "model": wl["model"], "global_batch": B * world,
                       "per_gpu_batch": B, "num_accum": res["num_accum"], "image": [H, W],
                       "parallelism": f"dp{world}", "reference_config": ref_cfg,
                       "matmul_precision": precision, "hipgraph": graph},
            "roofline": res.get("roofline"), "cpu_baseline": cpu, "loss": round(res["loss"], 5),
            "peak_mem_GB": res["peak_mem_GB"],
            "rccl_world": world if (world > 1 or args.ddp) else None,
        }
        if "allreduce" in res:
            line["allreduce"] = res["allreduce"]
        if files is not None:
            line["data_pipeline"] = files
        line.update(res.get("extra", {}))
        if secondary:
            line["secondary"] = secondary.pop("newcrfs_kitti", None)
            if secondary:
                line["secondaries"] = secondary
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
