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


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, grad_scale=1.0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.grad_scale = grad_scale
        self._tables = {}

    def _signature(self, plist):
        return tuple((p.data_ptr(), p.grad.data_ptr(), getattr(p, "_vit_shadow", None) is not None and
                      p._vit_shadow.data_ptr()) for p in plist)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            plist = [p for p in group["params"] if p.grad is not None]
            if not plist:
                continue
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
            # parameters are grouped by their step count (all equal in normal training)
            by_step = {}
            for p in plist:
                by_step.setdefault(int(self.state[p]["step"].item()), []).append(p)
            for step0, ps in by_step.items():
                for p in ps:
                    self.state[p]["step"] += 1
                t = step0 + 1
                b1, b2 = group["betas"]
                shadows = [getattr(p, "_vit_shadow", None) for p in ps]
                sdt = next((s.dtype for s in shadows if s is not None), torch.float32)
                shadows = [s if (s is not None and s.dtype == sdt) else None for s in shadows]
                key = (gi, step0 >= 0, self._signature(ps), sdt)
                tab = self._tables.get(key[:2])
                if tab is None or tab[0] != key:
                    entries = [(p, p.grad, self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"], s)
                               for p, s in zip(ps, shadows)]
                    for p, g, m, v, _ in entries:
                        for tt in (g, m, v):
                            if not tt.is_contiguous():
                                raise RuntimeError("FusedAdamW: non-contiguous grad/state")
                    dev_tab, n = _ops.build_chunk_table(entries, ps[0].device)
                    tab = (key, dev_tab, n)
                    self._tables[key[:2]] = tab
                _, dev_tab, n = tab
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
    """mean softmax cross-entropy (nn.CrossEntropyLoss() default) — fused HIP kernel, gradient precomputed."""
    return _XentFn.apply(logits, labels)


class CrossEntropyLoss(nn.Module):
    """Drop-in for nn.CrossEntropyLoss() as used by the reference (train.py:81): mean reduction, no weights."""

    def forward(self, logits, labels):
        return cross_entropy(logits, labels)
