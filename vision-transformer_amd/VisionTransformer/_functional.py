"""Module-level HIP autograd ops: what `Head`, `MultiHeadAttention`, `FeedForward`, `Block`, `TransformerEncoder` and
`PatchEmbedding` run when they are called on their own (the whole-model hot path goes through _engine instead).

Every op runs libvit_hip kernels; weights are fp32 masters cast to the activation dtype by the copy kernel.
Gradients flow through standard autograd into each parameter's `.grad`.
"""
import torch
import torch.nn.functional as F

from . import _cpu, _ops
from ._ops import ACT_NONE, ACT_RELU

DROPOUT_P = 0.2


def _cast(w, dtype):
    """fp32 master -> compute dtype, by the HIP copy kernel."""
    w = w.contiguous()
    if w.dtype == dtype:
        return w
    out = torch.empty(w.shape, dtype=dtype, device=w.device)
    n = w.numel()
    _ops.copy2d(w.view(1, n), n, out.view(1, n), n, 1, n)
    return out


def _flat2(x):
    return x.reshape(-1, x.shape[-1]).contiguous()


def _wgrad_into(dy2, x2, w):
    m, n, k = dy2.shape[1], x2.shape[1], dy2.shape[0]
    g = torch.empty(m, n, dtype=torch.float32, device=dy2.device)
    tiles = ((m + 127) // 128) * ((n + 127) // 128)
    split = max(1, min((1024 + tiles - 1) // tiles, max(1, k // 512), 32))
    _ops.gemm(dy2, x2, g, m, n, k, m, n, n, a_kcontig=False, b_kcontig=False, split_k=split)
    return g.view(w.shape)


class LinearFn(torch.autograd.Function):
    """y = act(x W^T + b) (nn.Linear, transformer.py:12-18,38,56,58 / vit.py:70,73); act in {none, relu}."""

    @staticmethod
    def forward(ctx, x, w, b, act):
        x2 = _flat2(x)
        wc = _cast(w, x2.dtype)
        y = _ops.linear(x2, wc, bias=None if b is None else b.float().contiguous(), act=act)
        ctx.save_for_backward(x2, w, y if act == ACT_RELU else None)
        ctx.act, ctx.has_b, ctx.xshape = act, b is not None, x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        dy2 = _flat2(dy)
        if dy2.dtype != x2.dtype:
            dy2 = _cast(dy2, x2.dtype)
        M, K = x2.shape
        N = w.shape[0]
        dx = db = dw = None
        g = _ops.relu_bwd(dy2, y) if ctx.act == ACT_RELU else dy2      # dy * (y > 0)
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, dtype=x2.dtype, device=x2.device)
            _ops.gemm(g, _cast(w, x2.dtype), dx, M, K, N, N, K, K, b_kcontig=False)
            dx = dx.view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            dw = _wgrad_into(g, x2, w)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = torch.empty(N, dtype=torch.float32, device=x2.device)
            _ops.colsum(g, M, N, N, db)
        return dx, dw, db, None


class LayerNormFn(torch.autograd.Function):
    """nn.LayerNorm(eps=1e-5) on the last dim (transformer.py:71-72)."""

    @staticmethod
    def forward(ctx, x, g, b):
        x2 = _flat2(x)
        y, mean, rstd = _ops.layernorm_fwd(x2, g.float().contiguous(), b.float().contiguous())
        ctx.save_for_backward(x2, g, mean, rstd)
        ctx.xshape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, g, mean, rstd = ctx.saved_tensors
        dy2 = _flat2(dy).to(x2.dtype)
        rows, cols = x2.shape
        dx = torch.empty_like(x2)
        part = _ops.layernorm_bwd(dy2, x2, g.float().contiguous(), mean, rstd, dx)
        dg = torch.empty(cols, dtype=torch.float32, device=x2.device)
        db = torch.empty(cols, dtype=torch.float32, device=x2.device)
        _ops.colsum(part[0], part.shape[1], cols, cols, dg)
        _ops.colsum(part[1], part.shape[1], cols, cols, db)
        return dx.view(ctx.xshape), dg, db


class DropoutFn(torch.autograd.Function):
    """Dropout(p) with counter-hash masks (train mode only); the backward regenerates the same mask."""

    @staticmethod
    def forward(ctx, x, p, seed):
        x = x.contiguous()
        y = torch.empty_like(x)
        _ops.dropout_bwd(x, y, p, seed)
        ctx.p, ctx.seed = p, seed
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        _ops.dropout_bwd(dy, dx, ctx.p, ctx.seed)
        return dx, None, None


def dropout(x, training, p=DROPOUT_P):
    if not training or p == 0.0:
        return x
    if not x.is_cuda:
        return F.dropout(x, p, True)                       # host path (_cpu.py)
    seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
    return DropoutFn.apply(x, p, seed)


# ---- device dispatch used by the module forwards: ROCm tensors run the HIP ops above, CPU tensors (model and
# input on the host, train.py --device cpu) run the host path.  A mixed call reaches the HIP op, which raises.
def _host(*ts):
    return all(t is None or not t.is_cuda for t in ts)


def linear(x, w, b, act):
    if _host(x, w, b):
        y = F.linear(x, w, b)
        return torch.relu(y) if act == ACT_RELU else y
    return LinearFn.apply(x, w, b, act)


def layer_norm(x, g, b):
    if _host(x, g, b):
        return F.layer_norm(x, (x.shape[-1],), g, b, 1e-5)
    return LayerNormFn.apply(x, g, b)


def head_attention(x, wq, wk, wv):
    if _host(x, wq, wk, wv):
        o, probs = _cpu.attention(x, torch.cat([wq, wk, wv], dim=0), 1, want_probs=True)
        return o, probs[:, 0].detach()
    return HeadAttentionFn.apply(x, wq, wk, wv)


def patch_embed(x, w, b, cls, pos, P, dtype):
    if _host(x, w, b, cls, pos):
        return _cpu.patch_embed(x, w, b, cls, pos, P)
    return PatchEmbedFn.apply(x, w, b, cls, pos, P, dtype)


class HeadAttentionFn(torch.autograd.Function):
    """One attention head (transformer.py:20-31): k, q, v projections (no bias), softmax(q k^T * sqrt(hd)) v.
    Returns (out, wei); `wei` is returned for inspection and is not differentiable."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv):
        B, T, D = x.shape
        hd = wq.shape[0]
        x2 = _flat2(x)
        dt = x2.dtype
        wpack = torch.empty(3 * hd, D, dtype=dt, device=x.device)
        for i, w in enumerate((wq, wk, wv)):
            _ops.copy2d(w.contiguous(), D, wpack[i * hd:(i + 1) * hd], D, hd, D)
        qkv = _ops.linear(x2, wpack)
        probs = torch.empty(B, 1, T, T, dtype=torch.float32, device=x.device)
        o32 = (torch.empty(B * T, hd, dtype=torch.float32, device=x.device)
               if _ops.attn_bwd_uses_o32(B, T, 1, hd, dt) else None)
        o, lse = _ops.attn_fwd(qkv, B, T, 1, hd, float(hd) ** 0.5, probs=probs, o32=o32)
        ctx.save_for_backward(x2, wpack, qkv, o, lse, o32)
        ctx.dims = (B, T, D, hd)
        wei = probs.view(B, T, T)
        ctx.mark_non_differentiable(wei)
        return o.view(B, T, hd), wei

    @staticmethod
    def backward(ctx, dout, _dwei):
        x2, wpack, qkv, o, lse, o32 = ctx.saved_tensors
        B, T, D, hd = ctx.dims
        d_o = _flat2(dout).to(x2.dtype)
        dqkv = _ops.attn_bwd(qkv, o, d_o, lse, B, T, 1, hd, float(hd) ** 0.5, o32=o32)
        dx = torch.empty(B * T, D, dtype=x2.dtype, device=x2.device)
        _ops.gemm(dqkv, wpack, dx, B * T, D, 3 * hd, 3 * hd, D, D, b_kcontig=False)
        dw = torch.empty(3 * hd, D, dtype=torch.float32, device=x2.device)
        _ops.gemm(dqkv, x2, dw, 3 * hd, D, B * T, 3 * hd, D, D, a_kcontig=False, b_kcontig=False)
        return dx.view(B, T, D), dw[:hd], dw[hd:2 * hd], dw[2 * hd:]


class PatchEmbedFn(torch.autograd.Function):
    """Conv2d(k=s=P) + flatten + permute + cat(CLS LAST) + pos (vit.py:21-29,39-42) as im2col + GEMM."""

    @staticmethod
    def forward(ctx, x, w, b, cls, pos, P, dtype):
        B = x.shape[0]
        D = w.shape[0]
        cols = _ops.im2col(x.contiguous(), P, dtype)
        N = cols.shape[0] // B
        T = N + 1
        wc = _cast(w.reshape(D, -1), dtype)
        x0 = torch.empty(B * T, D, dtype=dtype, device=x.device)
        _ops.gemm(cols, wc, x0, B * N, D, cols.shape[1], cols.shape[1], cols.shape[1], D, bias=b.float().contiguous(),
                  res=pos.reshape(T, D).float().contiguous(), ldres=D, res_rowmod=N, out_group=(N, T))
        _ops.embed_cls(cls.float().contiguous(), pos.float().contiguous(), x0, B, T, D)
        ctx.save_for_backward(cols)
        ctx.dims = (B, N, T, D, tuple(w.shape))
        return x0.view(B, T, D)

    @staticmethod
    def backward(ctx, dx):
        (cols,) = ctx.saved_tensors
        B, N, T, D, wshape = ctx.dims
        dx = dx.contiguous().view(B * T, D).to(cols.dtype)
        dcls = torch.empty(B, 1, D, dtype=torch.float32, device=dx.device)
        _ops.copy2d(dx[N:], T * D, dcls.view(B, D), D, B, D)
        dpos = torch.empty(1, T, D, dtype=torch.float32, device=dx.device)
        _ops.colsum(dx, B, T * D, T * D, dpos.view(-1))
        dpatch = torch.empty(B * N, D, dtype=dx.dtype, device=dx.device)
        _ops.copy2d(dx, D, dpatch, D, B * N, D, group=(N, T))
        db = torch.empty(D, dtype=torch.float32, device=dx.device)
        _ops.colsum(dpatch, B * N, D, D, db)
        dw = torch.empty(D, cols.shape[1], dtype=torch.float32, device=dx.device)
        _ops.gemm(dpatch, cols, dw, D, cols.shape[1], B * N, D, cols.shape[1], cols.shape[1], a_kcontig=False,
                  b_kcontig=False)
        return None, dw.view(wshape), db, dcls, dpos, None, None
