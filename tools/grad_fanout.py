"""Where autograd's gradient-accumulation adds come from in one NeW-CRFs-L07 train step: walk the
backward graph and count, per node type, the nodes whose output feeds more than one consumer (each
extra consumer is one torch add in backward).  Informational (profiles/r03_grad_fanout.txt).

  python tools/grad_fanout.py [--height 480 --width 640]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    a = ap.parse_args()
    from mdemi.model.NewCRFs import NewCRFDepth
    from mdemi.train import SILogLoss
    dev = torch.device("cuda", 0)
    m = NewCRFDepth(version="large07", max_depth=10.0).to(dev).train()
    img = torch.randn(1, 3, a.height, a.width, device=dev)
    gt = torch.rand(1, 1, a.height, a.width, device=dev) * 9 + 0.5
    loss = SILogLoss(10.0, 0.15)(m(img), gt)
    uses = collections.Counter()
    seen, stack = set(), [loss.grad_fn]
    while stack:
        n = stack.pop()
        if n is None or n in seen:
            continue
        seen.add(n)
        for nxt, slot in n.next_functions:
            if nxt is not None:
                uses[(nxt, slot)] += 1  # per output slot: two outputs of one node are not summed
                stack.append(nxt)
    fan = collections.Counter()
    for (n, _), u in uses.items():
        if u > 1 and type(n).__name__ != "AccumulateGrad":
            fan[type(n).__name__] += u - 1
    acc = sum(u - 1 for (n, _), u in uses.items() if u > 1 and type(n).__name__ == "AccumulateGrad")
    print(f"backward nodes {len(seen)}; extra consumers (=> accumulation adds) by producer node type:")
    for k, v in fan.most_common():
        print(f"  {v:4d}  {k}")
    print(f"  {acc:4d}  AccumulateGrad (parameters used more than once)")


if __name__ == "__main__":
    main()
