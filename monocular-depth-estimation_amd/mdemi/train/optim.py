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
    CUDA params; one gradient-norm kernel + one update kernel per step, no host sync.

    Each parameter keeps its own step count (torch's state[p]["step"]): a parameter
    whose gradient first appears at optimizer step k is bias-corrected as step 1 there.
    The counts live in a device int32 array (one slot per parameter, in param_groups
    order) that the update kernel reads and a trailing kernel advances; ``steps`` is the
    host mirror.

    capturable=True: the per-step hyperparameters (lr, betas) are read on the device
    from a schedule table (set_schedule; default: the groups' current values) indexed by
    a device step counter, so the whole step can live in a captured hipGraph
    (mdemi_adamw_step_dev).  The host mirrors (step_count, steps) are advanced by the
    caller after each replay (``replayed()``; Trainer does)."""

    def __init__(self, param_groups, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_grad_norm=0.0,
                 capturable=False):
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
        # every gradient is taken at grad_scale x its value, in the clip norm and the update
        # (Trainer sets 1/world when the data-parallel all-reduce leaves sums: the mean's
        # scale rides on this step instead of a separate sweep over the gradients)
        self.grad_scale = 1.0
        self.state = {}
        self.step_count = 0  # optimizer steps taken (the schedule position)
        self._slot = {}
        for p in (p for g in self.param_groups for p in g["params"]):
            self._slot.setdefault(p, len(self._slot))
        self.steps = [0] * len(self._slot)  # host mirror of the per-parameter step counters
        self._steps_dev = None
        self._chunk = L.load().mdemi_multi_tensor_chunk()
        self._sumsq = None
        self.capturable = bool(capturable)
        self._sched_rows = None  # host schedule [(lr, beta1, beta2, eps, wd) per group] per step
        self._sched_dev = None
        self._step_dev = None
        self._tbl_key = None
        self._tbl_slots = []
        # bumped whenever a device address the update reads may have changed (new state
        # tensors, a rebuilt pointer table): a captured graph recorded with an older
        # layout must be re-captured (Trainer checks)
        self.layout_version = 0
        # parameter -> persistent bf16 copy the update also writes (mdemi_adamw_step16): kept
        # for every parameter a bf16 GEMM has read (bf16 storage), so the next forward
        # finds a valid copy instead of casting each weight again
        self._b16 = {}

    # ---- capturable schedule ----
    def set_schedule(self, rows):
        """rows[s][g] = (lr, beta1, beta2, eps, weight_decay) used by optimizer step s (0-based)."""
        if not rows or any(len(r) != len(self.param_groups) for r in rows):
            raise ValueError("FusedAdamW.set_schedule: one row per step, one entry per parameter group")
        self._sched_rows = [[tuple(float(v) for v in e) for e in r] for r in rows]
        self._sched_dev = None
        self.layout_version += 1

    def _device_schedule(self, dev, taken):
        """taken: optimizer steps completed before the one being launched."""
        if self._sched_dev is None:
            rows = self._sched_rows
            if rows is None:  # constant hyperparameters: the groups' current values
                rows = [[(g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"])
                         for g in self.param_groups]]
            flat = [v for r in rows for e in r for v in (*e, 0.0)]  # mdemi_adamw_group: 5 floats + pad
            t = torch.tensor(flat, dtype=torch.float32)
            self._sched_dev = (t.to(dev), len(rows))
            if self._step_dev is None:
                self._step_dev = torch.full((1,), taken, dtype=torch.int32, device=dev)
            else:  # keep the address a captured graph recorded
                self._step_dev.fill_(taken)
        return self._sched_dev

    def zero_grad(self, set_to_none=True):
        for g in self.param_groups:
            for p in g["params"]:
                if set_to_none:
                    p.grad = None
                elif p.grad is not None:
                    p.grad.zero_()

    def _with_grad(self):
        return [p for g in self.param_groups for p in g["params"] if p.grad is not None]

    def _refs(self):
        refs, items_t, items_c, slots, p16 = [], [], [], [], []
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
                r.numel, r.group, r.step_slot = p.numel(), gi, self._slot[p]
                ti = len(refs)
                refs.append(r)
                slots.append(self._slot[p])
                b16 = self._b16.get(p)
                p16.append(b16.data_ptr() if b16 is not None else 0)
                nch = max(1, math.ceil(p.numel() / self._chunk))
                items_t.extend([ti] * nch)
                items_c.extend(range(nch))
        return refs, items_t, items_c, slots, p16

    def _key(self, params):
        """Every address the pointer table holds: a param, its grad, its state."""
        key = []
        for p in params:
            st = self.state.get(p)
            b16 = self._b16.get(p)
            key.append((p.data_ptr(), p.grad.data_ptr(),
                        st["exp_avg"].data_ptr() if st else 0, st["exp_avg_sq"].data_ptr() if st else 0,
                        b16.data_ptr() if b16 is not None else 0))
        return tuple(key)

    @torch.no_grad()
    def step(self):
        params = self._with_grad()
        if not params:
            return
        # the update writes the parameters through raw pointers: bf16 copies made before it
        # (functional.b16_of) are stale from here on
        from .. import functional as _mf
        for p in params:  # parameters a bf16 GEMM read this step get a maintained bf16 copy
            if p not in self._b16 and _mf._b16_rec(p, p.numel()) is not None:
                self._b16[p] = torch.empty(p.shape, dtype=torch.bfloat16, device=p.device)
        _mf.bump_weight_epoch()
        capturing = torch.cuda.is_current_stream_capturing()
        dev = torch.device("cuda", torch.cuda.current_device())
        lib = L.load()
        # device table of (param, grad, state) pointers: rebuilt only when an address moved
        # (set_to_none grads, replaced param storage, loaded state), so a step with
        # persistent tensors (captured graphs, DDP bucket views) issues no host->device copy
        key = self._key(params)
        if key != self._tbl_key:
            # inside a capture (gradients handed out by the captured backward) the upload is a
            # memcpy node from the pinned host table, which stays alive with the device copy:
            # every replay re-copies the same addresses
            refs, items_t, items_c, slots, p16 = self._refs()
            nt, ni = len(refs), len(items_t)
            raw = (L.TensorRef * nt)(*refs)
            rb = (ctypes.sizeof(raw) + 255) // 256 * 256
            pb = (8 * nt + 255) // 256 * 256 if any(p16) else 0  # bf16 copy pointers (mdemi_adamw_step16)
            wsb = lib.mdemi_grad_norm_workspace_size(ni)
            host = torch.empty(rb + pb + wsb, dtype=torch.uint8, pin_memory=True)
            ctypes.memmove(host.data_ptr(), ctypes.addressof(raw), ctypes.sizeof(raw))
            if pb:
                host[rb:rb + 8 * nt].view(torch.int64).copy_(torch.tensor(p16, dtype=torch.int64))
            w0 = rb + pb
            host[w0:w0 + 8 * ni].view(torch.int32).copy_(torch.tensor(items_t + items_c, dtype=torch.int32))
            dev_buf = host.to(dev, non_blocking=True)
            self._tbl = (host, dev_buf, dev_buf.data_ptr(), dev_buf.data_ptr() + w0, nt, ni,
                         dev_buf.data_ptr() + rb if pb else None)
            self._tbl_key = self._key(params)
            self._tbl_slots = slots
            self.layout_version += 1
        _, _, tl_ptr, ws_ptr, nt, ni, p16_ptr = self._tbl
        if self._steps_dev is None:
            if capturing:
                raise RuntimeError("FusedAdamW: step counters must exist before hipGraph capture")
            self._steps_dev = torch.tensor(self.steps, dtype=torch.int32).to(dev)
        if self._sumsq is None:
            self._sumsq = torch.zeros(1, device=dev, dtype=torch.float32)
        gs = float(self.grad_scale)
        if self.max_grad_norm > 0:
            L.check(lib.mdemi_grad_sumsq(tl_ptr, nt, ni, gs, self._sumsq.data_ptr(), ws_ptr, L.stream()), "grad_sumsq")
        clip = self._sumsq.data_ptr() if self.max_grad_norm > 0 else None
        steps_ptr = self._steps_dev.data_ptr()
        if self.capturable:
            sched, nsteps = self._device_schedule(dev, self.step_count)
            L.check(lib.mdemi_adamw_step_dev16(tl_ptr, nt, sched.data_ptr(), nsteps, len(self.param_groups),
                                               self._step_dev.data_ptr(), steps_ptr, clip, self.max_grad_norm, gs,
                                               ni, p16_ptr, ws_ptr, L.stream()), "adamw_step_dev")
        else:
            groups = (L.AdamWGroup * len(self.param_groups))()
            for i, g in enumerate(self.param_groups):
                groups[i].lr, (groups[i].beta1, groups[i].beta2) = g["lr"], g["betas"]
                groups[i].eps, groups[i].weight_decay = g["eps"], g["weight_decay"]
            L.check(lib.mdemi_adamw_step16(tl_ptr, nt, groups, len(self.param_groups), clip, self.max_grad_norm, gs,
                                           self.step_count + 1, steps_ptr, ni, p16_ptr, ws_ptr, L.stream()),
                    "adamw_step")
        for p, b16 in self._b16.items():  # the update wrote these copies at the new weight epoch
            if p.grad is not None:
                _mf.set_b16(p, b16)
        if not capturing:  # a capture records the step; replays advance the mirrors (replayed())
            self.replayed()

    def replayed(self):
        """Advance the host mirrors by one executed step over the current table's parameters."""
        self.step_count += 1
        for s in self._tbl_slots:
            self.steps[s] += 1

    def state_dict(self):
        """torch.optim.AdamW's layout: state keyed by each parameter's position across
        param_groups (not by the order gradients first appeared), a per-parameter "step",
        and "params" index lists per group -- so save_checkpoint files
        (common_utils.py:12-31 optimizer_state_dict) round-trip with torch's AdamW."""
        state, groups, idx = {}, [], 0
        for g in self.param_groups:
            ids = []
            for p in g["params"]:
                st = self.state.get(p)
                if st is not None:
                    state[idx] = {"step": torch.tensor(float(self.steps[self._slot[p]])), "exp_avg": st["exp_avg"],
                                  "exp_avg_sq": st["exp_avg_sq"]}
                ids.append(idx)
                idx += 1
            gd = {k: v for k, v in g.items() if k != "params"}
            gd.update(amsgrad=False, maximize=False, foreach=None, capturable=self.capturable,
                      differentiable=False, fused=None, params=ids)
            groups.append(gd)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        """Load torch.optim.AdamW's layout (or our own state_dict).  Existing state tensors
        and step counters are overwritten in place, so a captured train step keeps valid
        addresses; state for a parameter that had none bumps ``layout_version``."""
        if "param_groups" not in sd or any("params" not in g for g in sd["param_groups"]):
            raise ValueError("FusedAdamW.load_state_dict: expected torch.optim.AdamW's layout (per-group 'params' "
                             "index lists, per-parameter 'step'); optimizer states written by the round-1 "
                             "FusedAdamW (top-level 'step') are not supported -- re-save them with this version")
        params = [p for g in self.param_groups for p in g["params"]]
        if len(sd["param_groups"]) != len(self.param_groups):
            raise ValueError("loaded state dict has a different number of parameter groups")
        order = [i for sg in sd["param_groups"] for i in sg["params"]]
        if len(order) != len(params):
            raise ValueError("loaded state dict contains a parameter group that doesn't match the size of the "
                             "optimizer's group")
        pos = {int(i): params[k] for k, i in enumerate(order)}
        new_state, steps, fresh = {}, [0] * len(self.steps), False
        for i, v in sd["state"].items():
            p = pos[int(i)]
            old = self.state.get(p)
            ent = {}
            for k in ("exp_avg", "exp_avg_sq"):
                src = v[k].detach().to(p.device, torch.float32)
                if old is not None and old[k].shape == src.shape:
                    old[k].copy_(src)
                    ent[k] = old[k]
                else:
                    ent[k] = src.clone()
                    fresh = True
            new_state[p] = ent
            steps[self._slot[p]] = int(float(v.get("step", 0)))
        if fresh or set(new_state) != set(self.state):
            self.layout_version += 1
        self.state = new_state
        self.steps = steps
        self.step_count = max(steps) if steps else 0
        if self._steps_dev is not None:
            self._steps_dev.copy_(torch.tensor(steps, dtype=torch.int32))
        if self._step_dev is not None:
            self._step_dev.fill_(self.step_count)
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            g.update({k: v for k, v in sg.items() if k in ("lr", "betas", "eps", "weight_decay", "initial_lr",
                                                          "max_lr", "min_lr", "max_momentum", "base_momentum")})
        if self._sched_rows is None and self._sched_dev is not None:  # constant-hyperparameter table: refresh
            rows = [[(g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"]) for g in self.param_groups]]
            flat = [v for r in rows for e in r for v in (*e, 0.0)]
            self._sched_dev[0].copy_(torch.tensor(flat, dtype=torch.float32))


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

    def values(self, s, g):
        """(lr, beta1) of parameter group g after s scheduler steps."""
        start = 0.0
        for i, (end, lr0, lr1, m0, m1) in enumerate(self.phases):
            if s <= end or i == len(self.phases) - 1:
                pct = (s - start) / (end - start) if end > start else 0.0
                lr = self._cos(g[lr0], g[lr1], pct)
                b1 = self._cos(g[m0], g[m1], pct) if self.cycle_momentum else g["betas"][0]
                return lr, b1
            start = end

    def step(self):
        self.last_step += 1
        s = self.last_step
        if s > self.total:
            raise ValueError(f"OneCycleLR stepped {s} times; total_steps={self.total}")
        for g in self.opt.param_groups:
            g["lr"], b1 = self.values(s, g)
            g["betas"] = (b1, g["betas"][1])

    def state_dict(self):
        return {"last_step": self.last_step, "total": self.total}

    def load_state_dict(self, sd):
        self.set_position(int(sd["last_step"]))

    def set_position(self, s):
        """Resume: the schedule after s scheduler steps (the optimizer steps a checkpoint
        recorded), as if step() had been called s times since construction."""
        if not 0 <= s <= self.total:
            raise ValueError(f"OneCycleLR position {s} outside [0, {self.total}]")
        self.last_step = s - 1
        self.step()

    def hyper_table(self):
        """Row s = (lr, beta1, beta2, eps, weight_decay) per group after s scheduler steps,
        s = 0..total: FusedAdamW.set_schedule's rows for a captured train step (the optimizer
        and the scheduler step together, so row s serves optimizer step s)."""
        rows = []
        for s in range(self.total + 1):
            row = []
            for g in self.opt.param_groups:
                lr, b1 = self.values(s, g)
                row.append((lr, b1, g["betas"][1], g["eps"], g["weight_decay"]))
            rows.append(row)
        return rows

    def get_last_lr(self):
        return [g["lr"] for g in self.opt.param_groups]
