"""Multi-tensor AdamW on libmdemi (mdemi_grad_sumsq + mdemi_adamw_step) with
clip_grad_norm_ folded in, and a OneCycle schedule restating
torch.optim.lr_scheduler.OneCycleLR (cos anneal, cycle_momentum on beta1)
from the config keys scheduler.{pct_start,div_factor,final_div_factor}."""
from __future__ import annotations

import ctypes
import math

import torch

from .. import _lib as L


class FusedAdamW:
    """torch.optim.AdamW semantics (decoupled weight decay, amsgrad=False) for fp32
    CUDA params; one gradient-norm kernel + one update kernel per step, no host sync."""

    def __init__(self, param_groups, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_grad_norm=0.0):
        if isinstance(param_groups, torch.Tensor) or (isinstance(param_groups, (list, tuple)) and param_groups and
                                                      isinstance(param_groups[0], torch.Tensor)):
            param_groups = [{"params": list(param_groups)}]
        if hasattr(param_groups, "__next__"):
            param_groups = [{"params": list(param_groups)}]
        self.param_groups = []
        for g in param_groups:
            g = dict(g)
            g["params"] = [p for p in g["params"] if p.requires_grad]
            g.setdefault("lr", lr)
            g.setdefault("betas", betas)
            g.setdefault("eps", eps)
            g.setdefault("weight_decay", weight_decay)
            g["initial_lr"] = g.get("initial_lr", g["lr"])
            self.param_groups.append(g)
        if len(self.param_groups) > 4:
            raise ValueError("FusedAdamW: at most 4 parameter groups")
        self.max_grad_norm = float(max_grad_norm)
        self.state = {}
        self.step_count = 0
        self._chunk = L.load().mdemi_multi_tensor_chunk()
        self._sumsq = None

    def zero_grad(self, set_to_none=True):
        for g in self.param_groups:
            for p in g["params"]:
                if set_to_none:
                    p.grad = None
                elif p.grad is not None:
                    p.grad.zero_()

    def _refs(self):
        refs, items_t, items_c = [], [], []
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.is_contiguous()):
                    raise ValueError("FusedAdamW: params and grads must be contiguous fp32 CUDA tensors")
                st = self.state.get(p)
                if st is None:
                    st = {"exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p)}
                    self.state[p] = st
                r = L.TensorRef()
                r.param, r.grad = p.data_ptr(), p.grad.data_ptr()
                r.exp_avg, r.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                r.numel, r.group = p.numel(), gi
                ti = len(refs)
                refs.append(r)
                nch = max(1, math.ceil(p.numel() / self._chunk))
                items_t.extend([ti] * nch)
                items_c.extend(range(nch))
        return refs, items_t, items_c

    @torch.no_grad()
    def step(self):
        refs, items_t, items_c = self._refs()
        if not refs:
            return
        self.step_count += 1
        dev = torch.device("cuda", torch.cuda.current_device())
        nt, ni = len(refs), len(items_t)
        lib = L.load()
        # one host->device copy per step: [TensorRef x nt | chunk_tensor | chunk_index | partials]
        raw = (L.TensorRef * nt)(*refs)
        rb = (ctypes.sizeof(raw) + 255) // 256 * 256
        wsb = lib.mdemi_grad_norm_workspace_size(ni)
        host = torch.empty(rb + wsb, dtype=torch.uint8, pin_memory=True)
        ctypes.memmove(host.data_ptr(), ctypes.addressof(raw), ctypes.sizeof(raw))
        host[rb:rb + 8 * ni].view(torch.int32).copy_(torch.tensor(items_t + items_c, dtype=torch.int32))
        dev_buf = host.to(dev, non_blocking=True)
        tl_ptr, ws_ptr = dev_buf.data_ptr(), dev_buf.data_ptr() + rb
        if self._sumsq is None:
            self._sumsq = torch.zeros(1, device=dev, dtype=torch.float32)
        if self.max_grad_norm > 0:
            L.check(lib.mdemi_grad_sumsq(tl_ptr, nt, ni, self._sumsq.data_ptr(), ws_ptr, L.stream()), "grad_sumsq")
        groups = (L.AdamWGroup * len(self.param_groups))()
        for i, g in enumerate(self.param_groups):
            groups[i].lr, (groups[i].beta1, groups[i].beta2) = g["lr"], g["betas"]
            groups[i].eps, groups[i].weight_decay = g["eps"], g["weight_decay"]
        L.check(lib.mdemi_adamw_step(tl_ptr, nt, groups, len(self.param_groups),
                                     self._sumsq.data_ptr() if self.max_grad_norm > 0 else None,
                                     self.max_grad_norm, self.step_count, ni, ws_ptr, L.stream()), "adamw_step")
        self._keepalive = (host, dev_buf)

    def state_dict(self):
        return {"step": self.step_count,
                "state": {i: v for i, v in enumerate(self.state.values())},
                "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]}

    def load_state_dict(self, sd):
        self.step_count = sd["step"]
        params = [p for g in self.param_groups for p in g["params"]]
        for i, v in sd["state"].items():
            self.state[params[int(i)]] = {k: t.to(params[int(i)].device) for k, t in v.items()}
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            g.update({k: v for k, v in sg.items()})


class OneCycleLR:
    """torch.optim.lr_scheduler.OneCycleLR (anneal_strategy='cos', three_phase=False,
    cycle_momentum=True on beta1 between base_momentum=0.85 and max_momentum=0.95)."""

    def __init__(self, optimizer, max_lr, total_steps, pct_start=0.3, div_factor=25.0, final_div_factor=1e4,
                 cycle_momentum=True, base_momentum=0.85, max_momentum=0.95):
        self.opt = optimizer
        self.total = int(total_steps)
        max_lrs = max_lr if isinstance(max_lr, (list, tuple)) else [max_lr] * len(optimizer.param_groups)
        for g, m in zip(optimizer.param_groups, max_lrs):
            g["initial_lr"] = m / div_factor
            g["max_lr"] = m
            g["min_lr"] = g["initial_lr"] / final_div_factor
            if cycle_momentum:
                g["betas"] = (max_momentum, g["betas"][1])
                g["max_momentum"], g["base_momentum"] = max_momentum, base_momentum
        self.cycle_momentum = cycle_momentum
        self.phases = [(float(pct_start * self.total) - 1, "initial_lr", "max_lr", "max_momentum", "base_momentum"),
                       (float(self.total - 1), "max_lr", "min_lr", "base_momentum", "max_momentum")]
        self.last_step = -1
        self.step()

    @staticmethod
    def _cos(start, end, pct):
        return end + (start - end) / 2.0 * (math.cos(math.pi * pct) + 1)

    def step(self):
        self.last_step += 1
        s = self.last_step
        if s > self.total:
            raise ValueError(f"OneCycleLR stepped {s} times; total_steps={self.total}")
        for g in self.opt.param_groups:
            start = 0.0
            for i, (end, lr0, lr1, m0, m1) in enumerate(self.phases):
                if s <= end or i == len(self.phases) - 1:
                    pct = (s - start) / (end - start) if end > start else 0.0
                    g["lr"] = self._cos(g[lr0], g[lr1], pct)
                    if self.cycle_momentum:
                        g["betas"] = (self._cos(g[m0], g[m1], pct), g["betas"][1])
                    break
                start = end

    def get_last_lr(self):
        return [g["lr"] for g in self.opt.param_groups]
