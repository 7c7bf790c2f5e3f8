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
    `.item()` or `+= 1` on the step path.  Device chunk tables are cached per group and keyed on every pointer they
    hold (param, grad, shadow, exp_avg, exp_avg_sq), and hold references to those tensors."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, grad_scale=1.0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.grad_scale = grad_scale
        self._tables = {}
        self._steps = {}          # group index -> (steps tensor [n] f32 CPU, host list of ints)

    # ---- step counters ------------------------------------------------------------------------------------------
    def _step_state(self, gi, group):
        ent = self._steps.get(gi)
        ps = group["params"]
        if ent is not None and len(ent[1]) == len(ps):
            return ent
        host = [int(float(self.state[p]["step"])) if "step" in self.state[p] else 0 for p in ps]
        buf = torch.tensor(host, dtype=torch.float32)
        for i, p in enumerate(ps):
            if "step" in self.state[p]:
                self.state[p]["step"] = buf[i]
        ent = (buf, host)
        self._steps[gi] = ent
        return ent

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._tables = {}         # the moments are new tensors: every cached chunk table is stale
        self._steps = {}

    def _signature(self, plist):
        st = self.state
        return tuple((p.data_ptr(), p.grad.data_ptr(),
                      shadow_of(p) is not None and shadow_of(p).data_ptr(),
                      st[p]["exp_avg"].data_ptr(), st[p]["exp_avg_sq"].data_ptr()) for p in plist)

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
                self._steps.pop(gi, None)
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
                shadows = [shadow_of(p) for p in ps]
                sdt = next((s.dtype for s in shadows if s is not None), torch.float32)
                shadows = [s if (s is not None and s.dtype == sdt) else None for s in shadows]
                key = (gi, len(by_step) == 1 or t)
                sig = (self._signature(ps), sdt)
                tab = self._tables.get(key)
                if tab is None or tab[0] != sig:
                    entries = [(p, p.grad, self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"], s)
                               for p, s in zip(ps, shadows)]
                    for p, g, m, v, _ in entries:
                        for tt in (g, m, v):
                            if not tt.is_contiguous():
                                raise RuntimeError("FusedAdamW: non-contiguous grad/state")
                    dev_tab, n = _ops.build_chunk_table(entries, ps[0].device)
                    tab = (sig, dev_tab, n, entries)          # entries keep every tabled tensor alive
                    self._tables[key] = tab
                _, dev_tab, n, _ = tab
                _ops.adamw(dev_tab, n, group["lr"], b1, b2, group["eps"], group["weight_decay"], 1.0 - b1 ** t,
                           1.0 - b2 ** t, self.grad_scale, sdt)
        return loss


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
