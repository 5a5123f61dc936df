"""Data-parallel gradient exchange (restated: the reference wraps its model in
DistributedDataParallel inside the missing run.py; evidence
utils/common_utils.py:20-21).  One process per GPU; the only exchange step of
a train step is the mean of every parameter gradient across ranks.

GradAllReduce packs gradients into ~bucket_mb buckets in reverse registration
order (the order backward produces them), and launches each bucket's
all-reduce from a post-accumulate-grad hook as soon as its last gradient
lands, so RCCL (torch.distributed "nccl" == RCCL over xGMI on ROCm) overlaps
the rest of the backward.  finish() waits for the outstanding collectives and
scatters bucket / world back into the .grad tensors.  The pack / unpack
sweeps are libmdemi kernels (copy2d / AXPBY); the CPU gloo tests swap them
for torch ops through the two hooks below, nothing else changes."""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradAllReduce:
    def __init__(self, model, bucket_mb: float = 64.0, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.buckets, cur, size = [], [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_mb * 2 ** 20:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.bucket_of = {p: bi for bi, b in enumerate(self.buckets) for p in b}
        self.launch_order: list[int] = []
        self._flat = [None] * len(self.buckets)
        self._works = []
        self._handles = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]
        self.reset()

    # ---- pack / unpack (libmdemi sweeps on the GPU) ----
    def _flatten(self, grads):
        from .. import functional as mf
        return mf.concat_channels([g.reshape(1, -1) for g in grads]).view(-1)

    def _unflatten_mean(self, flat, grads):
        from .. import _lib as L
        off = 0
        for g in grads:
            n = g.numel()
            L.call("mdemi_elementwise", L.EW_AXPBY, flat[off:off + n].data_ptr(), flat[off:off + n].data_ptr(),
                   g.data_ptr(), n, 1.0 / self.world, 0.0, L.stream())
            off += n

    # ---- protocol ----
    def reset(self):
        self._pending = [len(b) for b in self.buckets]
        self._works = []
        self.launch_order = []

    def _hook(self, p):
        bi = self.bucket_of[p]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            grads = [q.grad for q in self.buckets[bi]]
            flat = self._flatten(grads)
            self._flat[bi] = (flat, grads)
            self.launch_order.append(bi)
            self._works.append(dist.all_reduce(flat, group=self.group, async_op=True))

    def finish(self):
        if any(n != 0 for n in self._pending):
            missing = [bi for bi, n in enumerate(self._pending) if n != 0]
            raise RuntimeError(f"GradAllReduce: buckets {missing} never completed (unused parameters?)")
        for w in self._works:
            w.wait()
        for item in self._flat:
            if item is not None:
                self._unflatten_mean(*item)
        self._flat = [None] * len(self.buckets)
        self.last_launch_order = list(self.launch_order)
        self.reset()

    def remove(self):
        for h in self._handles:
            h.remove()


def broadcast_parameters(model, src: int = 0, group=None):
    """Identical replicas before the first step (what DDP's constructor does)."""
    with torch.no_grad():
        for t in model.state_dict().values():
            dist.broadcast(t, src, group=group)
