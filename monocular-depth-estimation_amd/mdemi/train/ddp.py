"""Data-parallel gradient exchange (restated: the reference wraps its model in
DistributedDataParallel inside the missing run.py; evidence
utils/common_utils.py:20-21).  One process per GPU; the only exchange step of
a train step is the mean of every parameter gradient across ranks.

Layout.  Parameters are grouped into ~bucket_mb buckets in reverse
registration order (the order backward produces their gradients).  Each
bucket is ONE persistent flat fp32 buffer, allocated once, and every
parameter's ``.grad`` is a view into its bucket (DDP's
``gradient_as_bucket_view``): autograd accumulates straight into the bucket,
so there is no pack and no unpack sweep, gradient accumulation over
``train.num_accum`` micro-steps happens in place, and the optimizer and a
captured hipGraph see the same gradient addresses every step.

Protocol.  A post-accumulate-grad hook counts the gradients that landed in
each bucket; a bucket is ready when all of them have.  Buckets are launched
strictly in index order (bucket i waits until buckets 0..i-1 have launched),
so every rank issues the same sequence of collectives whatever order its
autograd engine fires hooks in.  Each launch is an async all-reduce (SUM) on
torch.distributed's communication stream — backend "nccl" is RCCL over xGMI
on ROCm — overlapping the rest of the backward.  ``finish()`` waits for the
outstanding collectives and scales each bucket by 1/world in place (one
libmdemi sweep per bucket) -- unless ``scale_in_finish`` is off: mdemi's
Trainer folds 1/world into the optimizer step instead (FusedAdamW.grad_scale),
so the reduced sums are never swept just to be scaled.  Inside ``no_sync()`` the hooks only let
gradients accumulate; the reduction happens on the first backward outside it.

If something replaced a ``.grad`` (``zero_grad(set_to_none=True)``, a first
step before the views were installed), the hook copies it into the bucket
slice and re-installs the view, so the protocol stays correct.

Bucket rebuild (``rebuild_buckets``, on by default; torch DDP rebuilds its buckets after the
first iteration for the same reason).  Reverse registration order is only a guess at the
order backward produces gradients: a parameter registered early but used late (NeW-CRFs'
backbone out-norms, read by the decoder) finishes its bucket late, and strict index order
then holds every later bucket back (bench.py --ddp measured bucket 4 of the large07 NYU
step ready 8 ms before the end of backward, holding back 9 buckets that were ready 18-62 ms
earlier).  The first synchronised backward records the order the gradients actually land
in; ``finish()`` then regroups the parameters in that order (rank 0's order, broadcast, so
every rank builds the same buckets) and moves the reduced gradients into the new buffers.
From the second step on, buckets become ready in index order."""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist


class GradAllReduce:
    SLOT_ALIGN = 64  # elements

    def __init__(self, model, bucket_mb: float = 64.0, group=None, rebuild_buckets: bool = True):
        self.group = group
        self.bucket_mb = bucket_mb
        # finish() turns the sums into means in place; a consumer that applies 1/world itself
        # (FusedAdamW.grad_scale, wired by Trainer) sets this False and saves that sweep
        self.scale_in_finish = True
        self.world = dist.get_world_size(group)
        self.params = [p for p in model.parameters() if p.requires_grad]
        if not self.params:
            raise ValueError("GradAllReduce: model has no trainable parameters")
        dtype = self.params[0].dtype
        dev = self.params[0].device
        if any(p.dtype != dtype or p.device != dev for p in self.params):
            raise ValueError("GradAllReduce: all parameters must share one dtype and device")
        self._layout(list(reversed(self.params)))
        self._install_views(copy_existing=True)
        self._pindex = {p: i for i, p in enumerate(self.params)}
        self._rebuild = rebuild_buckets
        self._arrivals: list[int] = []  # parameter indices in gradient-arrival order (first synced backward)
        self.rebuilt = False
        self.launch_order: list[int] = []
        self.last_launch_order: list[int] = []
        self._works = []
        self._sync = True
        # trace_events: record a HIP event on the compute stream when each bucket becomes ready
        # (its last gradient landed) and when it is launched, and one at the end of backward
        # (finish) -- bench.py --ddp reports the offsets (eager steps only, never in a capture)
        self.trace_events = False
        self.trace = None
        self._handles = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]
        self.reset()

    def _layout(self, order):
        """Buckets of ~bucket_mb over the parameters in `order`, one zeroed flat buffer each."""
        self.buckets, cur, size = [], [], 0
        for p in order:
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= self.bucket_mb * 2 ** 20:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.bucket_of, self.slot = {}, {}
        self.flat = []
        for bi, b in enumerate(self.buckets):
            # every slot starts on a SLOT_ALIGN-element (256-B) boundary, so each .grad view
            # is as aligned as a fresh allocation and the vectorised sweeps over it (the norm,
            # AdamW) never fall back to scalar paths; the gaps are zero and stay zero
            off = 0
            for p in b:
                self.bucket_of[p] = bi
                self.slot[p] = (off, p.numel())
                off += -(-p.numel() // self.SLOT_ALIGN) * self.SLOT_ALIGN
            self.flat.append(torch.zeros(off, dtype=self.params[0].dtype, device=self.params[0].device))
        self.bucket_bytes = [f.numel() * f.element_size() for f in self.flat]

    def _rebuild_from_arrivals(self):
        """Regroup the buckets in the recorded arrival order (rank 0's), keeping the gradients."""
        seen = set(self._arrivals)
        order = self._arrivals + [i for i in reversed(range(len(self.params))) if i not in seen]
        self._arrivals = []
        self._rebuild = False
        t = torch.tensor(order, dtype=torch.int64, device=self.flat[0].device)
        if self.world > 1:
            dist.broadcast(t, 0, group=self.group)
        order = [int(i) for i in t.tolist()]
        pos = {pi: k for k, pi in enumerate(order)}
        done = [max(pos[self._pindex[p]] for p in b) for b in self.buckets]  # when each bucket completed
        if all(a < b for a, b in zip(done, done[1:])):
            return  # already ready in index order (the order inside a bucket does not matter)
        grads = {p: self._view(p) for p in self.params}  # views into the old buffers (kept alive here)
        self._layout([self.params[i] for i in order])
        for p in self.params:
            v = self._view(p)
            self._copy(grads[p], v)
            p.grad = v
        self.rebuilt = True

    # ---- gradient storage ----
    def _view(self, p):
        off, n = self.slot[p]
        return self.flat[self.bucket_of[p]][off:off + n].view_as(p)

    def _install_views(self, copy_existing=False):
        for p in self.params:
            v = self._view(p)
            if copy_existing and p.grad is not None:
                self._copy(p.grad, v)
            p.grad = v

    def _is_view(self, p):
        g = p.grad
        return g is not None and g.data_ptr() == self._view(p).data_ptr()

    # ---- device sweeps (libmdemi on the GPU; the CPU gloo tests override these two) ----
    def _copy(self, src, dst):
        if src.is_cuda:
            from .. import _lib as L
            s = src.contiguous()
            L.call("mdemi_elementwise", L.EW_AXPBY, s.data_ptr(), s.data_ptr(), dst.data_ptr(), s.numel(), 1.0, 0.0,
                   L.stream())
        else:
            dst.copy_(src)

    def _scale(self, flat, s):
        if flat.is_cuda:
            from .. import _lib as L
            L.call("mdemi_elementwise", L.EW_AXPBY, flat.data_ptr(), flat.data_ptr(), flat.data_ptr(), flat.numel(),
                   float(s), 0.0, L.stream())
        else:
            flat.mul_(s)

    # ---- protocol ----
    def reset(self):
        self._pending = [len(b) for b in self.buckets]
        self._next = 0
        self._works = []
        self.launch_order = []
        tracing = (self.trace_events and self.flat[0].is_cuda
                   and not torch.cuda.is_current_stream_capturing())
        self._trace = ({"ready": [None] * len(self.buckets), "launch": [None] * len(self.buckets),
                        "ready_order": [], "end": None} if tracing else None)

    def trace_offsets(self):
        """After a traced step (trace_events on; call after synchronising): per bucket, the ms
        from its readiness and from its launch to the end of backward, its bytes, and the
        order buckets became ready in."""
        tr = self.trace
        if tr is None or tr["end"] is None:
            return None
        end = tr["end"]
        rows = [{"bucket": i, "bytes": self.bucket_bytes[i],
                 "ready_before_end_ms": round(tr["ready"][i].elapsed_time(end), 3),
                 "launch_before_end_ms": round(tr["launch"][i].elapsed_time(end), 3)}
                for i in range(len(self.buckets))]
        return {"buckets": rows, "ready_order": list(tr["ready_order"])}

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (train.num_accum micro-steps); reduce on the next
        backward outside this context (torch DDP's no_sync)."""
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev

    def _hook(self, p):
        if not self._is_view(p):  # .grad was replaced: fold it back into the bucket
            g = p.grad
            self._copy(g, self._view(p))
            p.grad = self._view(p)
        if not self._sync:
            return
        if self._rebuild:
            self._arrivals.append(self._pindex[p])
        bi = self.bucket_of[p]
        self._pending[bi] -= 1
        if self._trace is not None and self._pending[bi] == 0:
            self._trace["ready"][bi] = self._event()
            self._trace["ready_order"].append(bi)
        # launch every ready bucket in index order (identical collective sequence on all ranks)
        while self._next < len(self.buckets) and self._pending[self._next] == 0:
            bi = self._next
            self.launch_order.append(bi)
            if self._trace is not None:
                self._trace["launch"][bi] = self._event()
            self._works.append(dist.all_reduce(self.flat[bi], group=self.group, async_op=True))
            self._next += 1

    @staticmethod
    def _event():
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        return e

    def finish(self):
        """Wait for the bucket all-reduces and turn the sums into means (in place)."""
        if any(n != 0 for n in self._pending):
            missing = [bi for bi, n in enumerate(self._pending) if n != 0]
            raise RuntimeError(f"GradAllReduce: buckets {missing} never completed (unused parameters?)")
        if self._trace is not None:
            self._trace["end"] = self._event()
            self.trace = self._trace
        for w in self._works:
            w.wait()
        if self.world > 1 and self.scale_in_finish:
            for flat in self.flat:
                self._scale(flat, 1.0 / self.world)
        for p in self.params:  # an optimizer may have replaced a view meanwhile
            if not self._is_view(p):
                p.grad = self._view(p)
        self.last_launch_order = list(self.launch_order)
        if self._rebuild and self._arrivals and not (self.flat[0].is_cuda and torch.cuda.is_current_stream_capturing()):
            self._rebuild_from_arrivals()
        self.reset()

    def zero_grad(self):
        """Zero the buckets (the gradients stay views; use instead of set_to_none)."""
        for flat in self.flat:
            flat.zero_()
        for p in self.params:
            if not self._is_view(p):
                p.grad = self._view(p)

    def allreduce_all(self):
        """All buckets reduced back to back with no overlap (bench: isolated comm cost)."""
        for flat in self.flat:
            dist.all_reduce(flat, group=self.group)

    def remove(self):
        for h in self._handles:
            h.remove()


def broadcast_parameters(model, src: int = 0, group=None):
    """Identical replicas before the first step (what DDP's constructor does)."""
    with torch.no_grad():
        for t in model.state_dict().values():
            dist.broadcast(t, src, group=group)
    from .. import functional as mf
    mf.bump_weight_epoch()  # the collective wrote the parameters: any bf16 copy is stale
