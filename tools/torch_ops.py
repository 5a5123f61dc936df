"""Which torch (non-libmdemi) device ops one train step of a bench workload issues, and from
where: torch.profiler over one step after warm-up, aten ops that launch device work grouped by
(op, innermost mdemi/ model source frame).   python tools/torch_ops.py [--model newcrfs]"""
import collections
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

OPS = ("aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::copy_", "aten::mul", "aten::mul_",
       "aten::sum", "aten::zeros", "aten::zeros_like", "aten::clone", "aten::contiguous", "aten::cat",
       "aten::div", "aten::sub", "aten::neg", "aten::index", "aten::where", "aten::masked_fill")


def main():
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
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        trainer.step(batches)
        torch.cuda.synchronize()
    by = collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        frames = [f for f in (ev.stack or []) if "mdemi" in f or "model/" in f or "train/" in f]
        where = frames[0] if frames else (ev.stack[0] if ev.stack else "?")
        shapes = ev.input_shapes[0] if ev.input_shapes else None
        by[(ev.name, where, str(shapes)[:40])] += 1
    for (name, where, shp), n in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f"{n:4d}  {name:18s} {shp:42s} {where}")


if __name__ == "__main__":
    main()
