"""Where one train step of a bench workload calls given libmdemi entry points from: every
_lib.call / direct lib call of the named entry points during one eager step (after warm-up)
is counted by (entry, first model / functional frames).
   python tools/call_sites.py --model depthformer_bf16 [entries=mdemi_cast_bf16,mdemi_colsum_f32]"""
import collections
import copy
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from mdemi import _lib as L  # noqa: E402


def site():
    fr = [f for f in traceback.extract_stack()[:-2] if "/mdemi/" in f.filename and "_lib.py" not in f.filename]
    fr = fr[::-1]
    keep = fr[:3] + [f for f in fr[3:8] if "functional.py" not in f.filename]
    return " < ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in keep)


def main():
    entries = set(os.environ.get("ENTRIES", "mdemi_cast_bf16,mdemi_colsum_f32").split(","))
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
    trainer = build_from_config(opt, device=dev, precision=precision)  # eager (no graph): Python sees every call
    batches = [bench.synthetic_batch(B, H, W, dev, seed=1000 + i, data_type=opt["dataset"]["data_type"])
               for i in range(trainer.num_accum)]
    for _ in range(2):
        trainer.step(batches)
    torch.cuda.synchronize()
    counts, elems = collections.Counter(), collections.Counter()
    lib = L.load()
    wrapped = {}
    for name in entries:
        fn = getattr(lib, name)

        def w(*a, _fn=fn, _n=name):
            k = (_n, site())
            counts[k] += 1
            if _n == "mdemi_cast_bf16":
                elems[k] += int(a[2])
            return _fn(*a)
        wrapped[name] = fn
        setattr(lib, name, w)
    try:
        trainer.step(batches)
        torch.cuda.synchronize()
    finally:
        for name, fn in wrapped.items():
            setattr(lib, name, fn)
    for (name, where), n in sorted(counts.items(), key=lambda kv: (-elems[kv[0]], -kv[1])):
        print(f"{n:4d} {elems[(name, where)] / 1e6:8.2f} M  {name:18s} {where}")


if __name__ == "__main__":
    main()
