"""Fused optimizer and loss for the training step (train.py:66,81,93,96).

FusedAdamW: torch.optim.AdamW semantics (decoupled weight decay, bias-corrected moments, amsgrad off) in ONE
multi-tensor HIP launch over every parameter; the same kernel refreshes the compute-dtype shadow weights the fused
engine reads (bf16 copies of the fp32 masters), so no separate cast pass runs per step.  The optimizer state keys
('step', 'exp_avg', 'exp_avg_sq') are those of torch.optim.AdamW, so `optimizer.state_dict()` checkpoints are
interchangeable with the reference's (train.py:73,110).

CrossEntropyLoss: nn.CrossEntropyLoss() (mean) as one fused softmax + NLL + gradient kernel.
"""
import math

import torch
import torch.nn as nn

from . import _ops
from ._engine import shadow_of


class FusedAdamW(torch.optim.Optimizer):
    """Step bookkeeping stays on the host: each group's per-parameter 'step' entries are 0-d views of ONE CPU
    tensor (torch AdamW's state format, so `state_dict()` / `load_state_dict()` interchange with it), advanced by a
    single in-place add per step, with a host-side mirror of the counts for the bias corrections — no per-parameter
    `.item()` or `+= 1` on the step path.  Device chunk tables are cached per (group, step-count class) and hold
    references to every tensor whose pointer they carry.  A cached table is reused while the optimizer's version
    (bumped by load_state_dict / add_param_group / fresh state) is unchanged and every parameter still has the very
    same .grad tensor object, the same moment tensor objects and every parameter the storage it was tabled with, so
    `p.data = other` or a replaced moment tensor rebuilds the table by itself (one data_ptr() per parameter per step,
    no per-step pointer signature of gradients and moments)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, grad_scale=1.0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid AdamW hyper-parameters")
        self._version = 0
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.grad_scale = grad_scale
        self._tables = {}
        self._steps = {}          # group index -> (params list, steps tensor [n] f32 CPU, host list of ints)

    def invalidate(self):
        """Drop every cached chunk table and step mirror (parameters re-pointed outside any engine)."""
        self._version += 1
        self._tables = {}
        self._steps = {}

    # ---- step counters ------------------------------------------------------------------------------------------
    def _step_state(self, gi, group):
        ent = self._steps.get(gi)
        ps = group["params"]
        if ent is not None and len(ent[0]) == len(ps) and all(a is b for a, b in zip(ent[0], ps)):
            return ent[1], ent[2]
        host = [int(float(self.state[p]["step"])) if "step" in self.state[p] else 0 for p in ps]
        buf = torch.tensor(host, dtype=torch.float32)
        for i, p in enumerate(ps):
            if "step" in self.state[p]:
                self.state[p]["step"] = buf[i]
        self._steps[gi] = (list(ps), buf, host)
        return buf, host

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self.invalidate()         # the moments are new tensors: every cached chunk table is stale

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        if hasattr(self, "_tables"):
            self.invalidate()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            ps_all = group["params"]
            idx = [i for i, p in enumerate(ps_all) if p.grad is not None]
            if not idx:
                continue
            plist = [ps_all[i] for i in idx]
            fresh = False
            for p in plist:
                if not p.is_cuda or p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                    raise RuntimeError("FusedAdamW: parameters and grads must be float32 on a ROCm device")
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdamW does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    fresh = True
            if fresh:
                self.invalidate()
            buf, host = self._step_state(gi, group)
            # advance the counters: one in-place add on the shared tensor, host mirror in Python ints
            if len(idx) == len(ps_all):
                buf += 1
            else:
                buf[torch.tensor(idx)] += 1
            by_step = {}
            for i in idx:
                host[i] += 1
                by_step.setdefault(host[i], []).append(ps_all[i])
            b1, b2 = group["betas"]
            for t, ps in by_step.items():
                # one table for the whole group while every parameter has the same step count, else one per count
                key = (gi, "all") if len(by_step) == 1 else (gi, "t", t)
                tab = self._tables.get(key)
                if tab is not None and not self._table_valid(tab, ps):
                    tab = None
                if tab is None:
                    shadows = [shadow_of(p) for p in ps]
                    sdt = next((s.dtype for s in shadows if s is not None), torch.float32)
                    shadows = [s if (s is not None and s.dtype == sdt) else None for s in shadows]
                    entries = [(p, p.grad, self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"], s)
                               for p, s in zip(ps, shadows)]
                    for p, g, m, v, _ in entries:
                        for tt in (g, m, v):
                            if not tt.is_contiguous():
                                raise RuntimeError("FusedAdamW: non-contiguous grad/state")
                    dev_tab, n = _ops.build_chunk_table(entries, ps[0].device)
                    # entries keep every tabled tensor alive; the raw shadow list is what the identity check compares
                    tab = (self._version, list(ps), [p.grad for p in ps], [shadow_of(p) for p in ps], dev_tab, n,
                           sdt, entries, [p.data_ptr() for p in ps],
                           [(self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"]) for p in ps],
                           [p.grad.data_ptr() for p in ps])
                    self._tables[key] = tab
                dev_tab, n, sdt = tab[4], tab[5], tab[6]
                _ops.adamw(dev_tab, n, group["lr"], b1, b2, group["eps"], group["weight_decay"], 1.0 - b1 ** t,
                           1.0 - b2 ** t, self.grad_scale, sdt)
        return loss

    def _table_valid(self, tab, ps):
        """Same optimizer version, same parameters, every parameter still holds the same .grad tensor object and the
        same moment tensor objects as when the table was built, and no parameter's or gradient's storage moved (`p.data = ...`
        re-points storage without changing any object identity).  Two data_ptr() per parameter plus
        identity checks: this runs every step.  The engine's shadows change only when it rebuilds its buffers, and
        then every gradient view is a new object too."""
        ver, tps, grads, ptrs, moments, gptrs = tab[0], tab[1], tab[2], tab[8], tab[9], tab[10]
        if ver != self._version or len(tps) != len(ps):
            return False
        state = self.state
        for a, b, g, ptr, (m, v), gp in zip(tps, ps, grads, ptrs, moments, gptrs):
            # the gradient's storage too: `p.grad.data = t` / `p.grad.set_(...)` keep the .grad object
            if a is not b or a.grad is not g or a.data_ptr() != ptr or g.data_ptr() != gp:
                return False
            st = state[a]
            if st["exp_avg"] is not m or st["exp_avg_sq"] is not v:
                return False
        return True


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        loss, dlogits = _ops.softmax_xent(logits.contiguous().float(), labels.contiguous().long())
        ctx.save_for_backward(dlogits)
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        (dlogits,) = ctx.saved_tensors
        return dlogits * g, None


def cross_entropy(logits, labels):
    """mean softmax cross-entropy (nn.CrossEntropyLoss() default) — fused HIP kernel, gradient precomputed; host
    tensors (the CPU path) use torch's own."""
    if not logits.is_cuda:
        return nn.functional.cross_entropy(logits, labels)
    return _XentFn.apply(logits, labels)


def make_optimizer(params, lr=1e-4, weight_decay=1e-4, device="cuda"):
    """The reference's optimizer (train.py:66, AdamW(lr, weight_decay=1e-4)): FusedAdamW on a ROCm device,
    torch.optim.AdamW on the host path."""
    if torch.device(device).type == "cpu":
        return torch.optim.AdamW(params, lr=lr, weight_decay=weight_decay)
    return FusedAdamW(params, lr=lr, weight_decay=weight_decay)


class CrossEntropyLoss(nn.Module):
    """Drop-in for nn.CrossEntropyLoss() as used by the reference (train.py:81): mean reduction, no weights."""

    def forward(self, logits, labels):
        return cross_entropy(logits, labels)
