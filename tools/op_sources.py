"""Where a train step issues given libmdemi entry points from (default: the bf16 casts and the
dropout sweeps of the configs[4] Depthformer step): every call of the named C entries during
one eager step is attributed to the innermost frames under mdemi/ that led to it, with the
tensor size, so a producer that could have written the bf16 copy itself can be found.
   python tools/op_sources.py [--model depthformer_bf16] [entry ...]"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from mdemi import _lib as L  # noqa: E402


def main():
    import copy

    from mdemi.train import build_from_config
    entries = [a for a in sys.argv[1:] if not a.startswith("--")] or ["mdemi_cast_bf16", "mdemi_dropout_dev16",
                                                                         "mdemi_elementwise", "mdemi_colsum_f32"]
    model = "depthformer_bf16"
    if "--model" in sys.argv:
        model = sys.argv[sys.argv.index("--model") + 1]
        entries = [e for e in entries if e != model]
    wl = bench.WORKLOADS[model]
    opt = copy.deepcopy(wl["opt"])
    B = int(opt["dataloader"]["batch_size"])
    torch.manual_seed(0)
    trainer = build_from_config(opt, device=torch.device("cuda", 0), precision=wl.get("precision", "fp32"))
    batches = [bench.synthetic_batch(B, wl["h"], wl["w"], "cuda", seed=1000 + i,
                                     data_type=opt["dataset"]["data_type"]) for i in range(trainer.num_accum)]
    for _ in range(2):
        trainer.step(batches)
    torch.cuda.synchronize()
    lib = L.load()
    counts = collections.Counter()
    orig = {}
    for name in entries:
        fn = getattr(lib, name)
        orig[name] = fn

        def wrapped(*args, _fn=fn, _name=name):  # noqa: E306
            stack = [f for f in traceback.extract_stack()[:-1] if "/mdemi/" in f.filename]
            inner = [f for f in stack if not f.filename.endswith(("_lib.py",))][-4:]
            outer = [f for f in stack if not f.filename.endswith(("_lib.py", "functional.py"))][-2:]
            where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in (inner + outer)[::-1])
            counts[(_name, where)] += 1
            return _fn(*args)
        setattr(lib, name, wrapped)
    try:
        trainer.step(batches)
        torch.cuda.synchronize()
    finally:
        for name, fn in orig.items():
            setattr(lib, name, fn)
    for (name, where), n in sorted(counts.items(), key=lambda kv: (kv[0][0], -kv[1])):
        print(f"{n:4d}  {name:24s} {where}")


if __name__ == "__main__":
    main()
