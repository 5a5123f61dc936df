"""Is the train step host-bound?  Times, per step, the CPU time to enqueue the whole step
(train_step returning, no sync) against the wall time with the GPU drained, for the default
bench workload.  Enqueue ~= wall means the GPU waits on Python/ctypes launch overhead."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monocular-depth-estimation_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


class A:
    model = "newcrfs"


def main():
    dev = torch.device("cuda", 0)
    cfg = bench.WORKLOADS["newcrfs"]
    model, opt, loss_fn = bench.build(A, dev)
    img, gt = bench.synthetic_batch(cfg["batch"], cfg["h"], cfg["w"], dev, seed=1)
    for _ in range(3):
        bench.train_step(model, opt, loss_fn, img, gt)
    torch.cuda.synchronize()
    for _ in range(5):
        t0 = time.perf_counter()
        bench.train_step(model, opt, loss_fn, img, gt)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"enqueue {1e3 * (t1 - t0):7.2f} ms   wall {1e3 * (t2 - t0):7.2f} ms", flush=True)


if __name__ == "__main__":
    main()
