"""Tensor-level wrappers over the C-ABI (no autograd here).  Every function launches on the current HIP stream
(or `stream`) and returns immediately.  Shapes/dtypes are validated on the host; the kernels re-validate."""
import ctypes
import os

import torch

from . import _lib
from ._lib import ACT_GELU, ACT_NONE, ACT_RELU, BF16, F32, FLAG_SHARED_CUS, MASK4  # noqa: F401

_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dtype_code(t):
    try:
        return _DT[t.dtype if isinstance(t, torch.Tensor) else t]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype if isinstance(t, torch.Tensor) else t}; use float32 or bfloat16")


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("VisionTransformer HIP path: tensors must live on a ROCm device (got CPU tensor); "
                               "the CPU restatement under oracle/ is test infrastructure, not a fallback")


def mask4_bytes(m, n):
    """Bytes of a VIT_MASK4 bit mask of an [m][n] tensor (include/vit_hip.h)."""
    return 4 * ((m + 3) // 4) * ((n + 3) // 4)


def mask4_empty(m, n, device):
    return torch.empty(mask4_bytes(m, n), dtype=torch.uint8, device=device)


def gemm(a, b, c, m, n, k, lda, ldb, ldc, a_kcontig=True, b_kcontig=True, alpha=1.0, beta=0.0, bias=None,
         act=ACT_NONE, aux=None, ldaux=0, res=None, ldres=0, res_rowmod=0, dropout_p=0.0, seed=0, split_k=1,
         out_group=(0, 0), workspace=None, colsum_part=None, mask_out=None, drop_row_stride=1, shared_cus=False,
         drop_row0=0, stream=None):
    """C[i][j] = epi(alpha * sum_r A(i,r) B(j,r)); see include/vit_hip.h.  `shared_cus`: VIT_FLAG_SHARED_CUS (other
    kernels — RCCL collectives — may hold CUs meanwhile: no persistent grid).  `colsum_part` (f32, colsum_part_rows(m) x n)
    receives per-256-row-block column sums of C as stored — finish with colsum_finish.  `aux` may be a uint8 mask4
    tensor (the ReLU mask saved by the forward); `mask_out` (uint8, mask4_bytes(m, n)) receives C's mask4 (dropout
    keep bits when dropout_p > 0, else C > 0).  `drop_row_stride` S: output row i draws the dropout bits of row i*S of
    the full tensor (C = token-0 rows of it); `drop_row0` R0: row i draws those of row i + R0 (C = a row range of a
    larger tensor).  Returns c."""
    _need_cuda(a, b, c, bias, aux, res, colsum_part, mask_out)
    if a.dtype != b.dtype:
        raise TypeError("gemm: A and B dtypes differ")
    if bias is not None and bias.dtype != torch.float32:
        raise TypeError("gemm: bias must be float32")
    d = _lib.GemmDesc()
    d.a, d.b, d.c = a.data_ptr(), b.data_ptr(), c.data_ptr()
    d.lda, d.ldb, d.ldc = lda, ldb, ldc
    d.m, d.n, d.k = m, n, k
    d.a_kcontig, d.b_kcontig = int(a_kcontig), int(b_kcontig)
    d.in_dtype, d.out_dtype = dtype_code(a), dtype_code(c)
    d.alpha, d.beta = alpha, beta
    d.bias = None if bias is None else bias.data_ptr()
    d.act = act
    if aux is not None:
        if aux.dtype == torch.uint8:
            if aux.numel() < mask4_bytes(m, n):
                raise ValueError("gemm: mask4 aux too small")
            d.aux, d.ldaux, d.aux_dtype = aux.data_ptr(), 0, MASK4
        else:
            d.aux, d.ldaux, d.aux_dtype = aux.data_ptr(), ldaux, dtype_code(aux)
    if mask_out is not None:
        if mask_out.dtype != torch.uint8 or mask_out.numel() < mask4_bytes(m, n):
            raise ValueError("gemm: mask_out must be uint8 with >= mask4_bytes(m, n) elements")
        d.mask_out = mask_out.data_ptr()
    d.dropout_row_stride = drop_row_stride
    d.flags = FLAG_SHARED_CUS if shared_cus else 0
    d.dropout_row0 = drop_row0
    if res is not None:
        d.res, d.ldres, d.res_rowmod, d.res_dtype = res.data_ptr(), ldres, res_rowmod, dtype_code(res)
    d.dropout_p, d.dropout_seed = dropout_p, seed & 0xFFFFFFFF
    d.split_k = split_k
    d.out_group_rows, d.out_group_stride = out_group
    if colsum_part is not None:
        if colsum_part.dtype != torch.float32 or colsum_part.numel() < colsum_part_rows(m) * n:
            raise ValueError("gemm: colsum_part must be float32 with >= ceil(m/256)*n elements")
        d.colsum_part = colsum_part.data_ptr()
    # split-K slabs (split_k > 1), or the slabs of the split-K tail of the last partial round of tiles
    need = _lib.load().vit_gemm_workspace_bytes(ctypes.byref(d))
    if need > 0:
        if workspace is None or workspace.numel() * workspace.element_size() < need:
            workspace = torch.empty(need // 4 + 1, dtype=torch.float32, device=c.device)
            if stream is not None:
                workspace.record_stream(stream)      # freed on return: not reusable before `stream` is done with it
        d.workspace, d.workspace_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
    _lib.check(_lib.load().vit_gemm(ctypes.byref(d), _stream(stream)), "vit_gemm")
    return c


def colsum_part_rows(m):
    """Rows of a GEMM's colsum_part: one per 256-row block of C."""
    return (m + 255) // 256


def linear(x2d, w, bias=None, out_dtype=None, act=ACT_NONE, **kw):
    """y = act(x @ w^T + bias) for row-major x [M,K], w [N,K]."""
    M, K = x2d.shape
    N = w.shape[0]
    y = torch.empty(M, N, dtype=out_dtype or x2d.dtype, device=x2d.device)
    return gemm(x2d, w, y, M, N, K, x2d.stride(0), w.stride(0), N, bias=bias, act=act, **kw)


def im2col(x, P, dtype, stream=None, cols=None):
    _need_cuda(x)
    B, C, H, W = x.shape
    n = (H // P) * (W // P)
    cols = torch.empty(B * n, C * P * P, dtype=dtype, device=x.device) if cols is None else cols
    _lib.call("vit_im2col", _ptr(x), dtype_code(x), _ptr(cols), dtype_code(dtype), B, C, H, W, P, _stream(stream))
    return cols


def col2im(cols, x, P, stream=None):
    """Inverse of im2col for k = s = P (a permutation): x[B, C, H, W] <- cols[B*N, C*P*P] (input-image gradient)."""
    _need_cuda(cols, x)
    B, C, H, W = x.shape
    _lib.call("vit_col2im", _ptr(cols), dtype_code(cols), _ptr(x), dtype_code(x), B, C, H, W, P, _stream(stream))
    return x


def embed_cls(cls, pos, x0, B, T, D, stream=None):
    _lib.call("vit_embed_cls", _ptr(cls), _ptr(pos), _ptr(x0), dtype_code(x0), B, T, D, _stream(stream))


def layernorm_fwd(x2d, gamma, beta, y=None, eps=1e-5, stream=None, mean=None, rstd=None):
    _need_cuda(x2d, gamma, beta)
    rows, cols = x2d.shape
    y = torch.empty_like(x2d) if y is None else y
    mean = torch.empty(rows, dtype=torch.float32, device=x2d.device) if mean is None else mean
    rstd = torch.empty(rows, dtype=torch.float32, device=x2d.device) if rstd is None else rstd
    _lib.call("vit_layernorm_fwd", _ptr(x2d), x2d.stride(0), _ptr(gamma), _ptr(beta), _ptr(y), y.stride(0),
              _ptr(mean), _ptr(rstd), rows, cols, eps, dtype_code(x2d), _stream(stream))
    return y, mean, rstd


def layernorm_bwd_parts(rows, cols):
    return _lib.load().vit_layernorm_bwd_parts(rows, cols)


def layernorm_bwd(dy, x, gamma, mean, rstd, dx_out, dres=None, drop_out=None, drop_p=0.0, drop_seed=0,
                  partial=None, osum=False, drop_mask=None, stream=None):
    """dx_out = LN_bwd(dy) (+ dres); drop_out = dx_out * keep (UNSCALED: consumers multiply by 1/(1-p)); returns
    partial [2, parts, cols] f32 (dgamma / dbeta per workgroup) — [3, parts, cols] with `osum`: + the column sums of
    the gradient the next Linear sees (drop_out / (1-p) when given, else dx_out), i.e. its bias gradient.  Reduce
    with colsum_finish.  `drop_mask` (uint8 mask4): the keep bits saved by the forward, instead of the hash."""
    rows, cols = x.shape
    if drop_mask is not None and (drop_mask.dtype != torch.uint8 or drop_mask.numel() < mask4_bytes(rows, cols)):
        raise ValueError("layernorm_bwd: drop_mask must be uint8 with >= mask4_bytes(rows, cols) elements")
    parts = layernorm_bwd_parts(rows, cols)
    if partial is None:
        partial = torch.empty(3 if osum else 2, parts, cols, dtype=torch.float32, device=x.device)
    _lib.call("vit_layernorm_bwd", _ptr(dy), dy.stride(0), _ptr(x), x.stride(0), _ptr(gamma), _ptr(mean), _ptr(rstd),
              _ptr(dres), _ptr(dx_out), _ptr(drop_out), drop_p, drop_seed & 0xFFFFFFFF, _ptr(drop_mask), _ptr(partial),
              int(bool(osum)),
              rows, cols, dtype_code(x), _stream(stream))
    return partial


def attn_fwd(qkv, B, T, H, hd, scale, o=None, lse=None, probs=None, o32=None, max_wgs=0, stream=None):
    """o = softmax(scale Q K^T) V per head; `o32` (bf16 only): also store O unrounded (fp32) for attn_bwd's delta
    where attn_bwd_uses_o32() says the backward takes it.  `max_wgs` > 0: at most that many workgroups for the
    persistent ring forward, for this call only (0: automatic / the library option)."""
    _need_cuda(qkv)
    D = H * hd
    o = torch.empty(B * T, D, dtype=qkv.dtype, device=qkv.device) if o is None else o
    lse = torch.empty(B, H, T, dtype=torch.float32, device=qkv.device) if lse is None else lse
    _lib.call("vit_attn_fwd", _ptr(qkv), _ptr(o), _ptr(o32), _ptr(lse), _ptr(probs), B, T, H, hd, scale,
              dtype_code(qkv), int(max_wgs), _stream(stream))
    return o, lse


def attn_bwd_uses_o32(B, T, H, hd, dtype):
    """True when attn_bwd at this shape forms delta from the forward's fp32 O (the tiled T > 256 path); the fused
    T <= 256 backward forms it from P and dP itself and reads neither O nor o32."""
    return bool(_lib.load().vit_attn_bwd_uses_o32(B, T, H, hd, dtype_code(dtype)))


def attn_bwd_workspace_bytes(B, T, H, hd, dtype):
    return _lib.load().vit_attn_bwd_workspace_bytes(B, T, H, hd, dtype_code(dtype))


def attn_bwd(qkv, o, d_o, lse, B, T, H, hd, scale, dqkv=None, workspace=None, o32=None, shared_cus=False,
             stream=None):
    dqkv = torch.empty_like(qkv) if dqkv is None else dqkv
    need = attn_bwd_workspace_bytes(B, T, H, hd, qkv.dtype)
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty(max(need // 4, 1), dtype=torch.float32, device=qkv.device)
    _lib.call("vit_attn_bwd", _ptr(qkv), _ptr(o), _ptr(o32), _ptr(d_o), _ptr(lse), _ptr(dqkv), B, T, H, hd, scale,
              dtype_code(qkv), _ptr(workspace), FLAG_SHARED_CUS if shared_cus else 0, _stream(stream))
    return dqkv


def attn_fwd_row0(qkv, B, T, H, hd, scale, o=None, lse=None, stream=None):
    """Attention output row 0 of every image (vit_attn_fwd_row0): o rows b*T and lse[b][h][0] are written, the other
    rows / entries are left as they are (o and lse may be fresh, uninitialised tensors)."""
    _need_cuda(qkv)
    D = H * hd
    o = torch.empty(B * T, D, dtype=qkv.dtype, device=qkv.device) if o is None else o
    lse = torch.empty(B, H, T, dtype=torch.float32, device=qkv.device) if lse is None else lse
    _lib.call("vit_attn_fwd_row0", _ptr(qkv), _ptr(o), _ptr(lse), B, T, H, hd, scale, dtype_code(qkv), _stream(stream))
    return o, lse


def attn_bwd_row0(qkv, d_o0, ldo, dqkv, B, T, H, hd, scale, stream=None):
    """Backward of attn_fwd_row0 from the row-0 output gradients d_o0 (image b at row b, stride ldo): dQ row 0 and all
    of dK, dV into dqkv (dQ rows 1..T-1 untouched)."""
    _need_cuda(qkv, d_o0, dqkv)
    _lib.call("vit_attn_bwd_row0", _ptr(qkv), _ptr(d_o0), ldo, _ptr(dqkv), B, T, H, hd, scale,
              dtype_code(qkv), _stream(stream))
    return dqkv


def colsum(x, rows, cols, ldx, out, beta=0.0, workspace=None, alpha=1.0, stream=None):
    need = _lib.load().vit_colsum_workspace_bytes(rows, cols)
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty(max(need // 4, 1), dtype=torch.float32, device=x.device)
    _lib.call("vit_colsum", _ptr(x), ldx, dtype_code(x), rows, cols, _ptr(out), alpha, beta, _ptr(workspace),
              _stream(stream))
    return out


def colsum_finish(part, outs, beta=0.0, stream=None):
    """outs[s] = beta * outs[s] + sum_p part[s][p] (fixed order) for s < len(outs) <= 3 — the second stage of the
    column sums vit_gemm (colsum_part) and vit_layernorm_bwd produce.  part: [sets, nparts, cols] or [nparts, cols]."""
    p3 = part if part.dim() == 3 else part.unsqueeze(0)
    n = len(outs)
    if not 1 <= n <= min(3, p3.shape[0]):
        raise ValueError(f"colsum_finish: {n} outputs for {p3.shape[0]} partial sets")
    for t in outs:
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != p3.shape[2]:
            raise ValueError("colsum_finish: outputs must be contiguous float32 of length cols")
    ptrs = [_ptr(t) for t in outs] + [None] * (3 - n)
    _lib.call("vit_colsum_finish", _ptr(p3), p3.shape[1], p3.shape[2], n, *ptrs, beta, _stream(stream))
    return outs


def colsum_finish_batch(jobs, stream=None):
    """Several colsum_finish jobs [(part, outs, beta), ...] (<= 8) in one launch; each job's outputs are bitwise what
    colsum_finish(part, outs, beta) gives."""
    if not 1 <= len(jobs) <= 8:
        raise ValueError("colsum_finish_batch: 1..8 jobs")
    arr = (_lib.ColsumJob * len(jobs))()
    for i, (part, outs, beta) in enumerate(jobs):
        p3 = part if part.dim() == 3 else part.unsqueeze(0)
        n = len(outs)
        if not 1 <= n <= min(3, p3.shape[0]) or not p3.is_contiguous() or p3.dtype != torch.float32:
            raise ValueError(f"colsum_finish_batch: job {i}: {n} outputs for {p3.shape[0]} partial sets")
        for t in outs:
            if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != p3.shape[2]:
                raise ValueError("colsum_finish_batch: outputs must be contiguous float32 of length cols")
        arr[i].part, arr[i].nparts, arr[i].cols, arr[i].nsets = _ptr(p3), p3.shape[1], p3.shape[2], n
        for s_, t in enumerate(outs):
            arr[i].out[s_] = _ptr(t)
        arr[i].beta = beta
    _lib.call("vit_colsum_finish_batch", arr, len(jobs), _stream(stream))


def copy2d(src, lds, dst, ldd, rows, cols, group=(0, 0), beta=0.0, stream=None):
    _lib.call("vit_copy2d", _ptr(src), lds, dtype_code(src), _ptr(dst), ldd, dtype_code(dst), rows, cols, group[0],
              group[1], beta, _stream(stream))
    return dst


def dropout_bwd(x, y, p, seed, scale=None, stream=None):
    """y = x * keep * scale (scale defaults to 1/(1-p))."""
    scale = 1.0 / (1.0 - p) if scale is None else scale
    _lib.call("vit_dropout_bwd", _ptr(x), _ptr(y), dtype_code(x), x.numel(), p, seed & 0xFFFFFFFF, scale,
              _stream(stream))
    return y


def mask4_apply(x, y, mask, scale=1.0, stream=None):
    """y = x * mask4 bit * scale for 2-D x, y (any float dtypes, row strides allowed)."""
    _need_cuda(x, y, mask)
    rows, cols = x.shape
    if mask.dtype != torch.uint8 or mask.numel() < mask4_bytes(rows, cols) or tuple(y.shape) != (rows, cols):
        raise ValueError("mask4_apply: bad mask or output shape")
    _lib.call("vit_mask4_apply", _ptr(x), x.stride(0), dtype_code(x), _ptr(y), y.stride(0), dtype_code(y), _ptr(mask),
              rows, cols, scale, _stream(stream))
    return y


def relu_bwd(dy, y, dx=None, stream=None):
    dx = torch.empty_like(dy) if dx is None else dx
    _lib.call("vit_relu_bwd", _ptr(dy), _ptr(y), _ptr(dx), dtype_code(dy), dy.numel(), _stream(stream))
    return dx


def gelu_fwd(x, y=None, stream=None):
    y = torch.empty_like(x) if y is None else y
    _lib.call("vit_gelu_fwd", _ptr(x), _ptr(y), x.numel(), _stream(stream))
    return y


def gelu_bwd(x, dy, dx=None, stream=None):
    dx = torch.empty_like(x) if dx is None else dx
    _lib.call("vit_gelu_bwd", _ptr(x), _ptr(dy), _ptr(dx), x.numel(), _stream(stream))
    return dx


def softmax_xent(logits, labels, stream=None):
    """Returns (loss [1] f32, dlogits [rows, classes] f32 = d(mean loss)/dlogits)."""
    _need_cuda(logits, labels)
    rows, classes = logits.shape
    loss = torch.empty(1, dtype=torch.float32, device=logits.device)
    dlogits = torch.empty_like(logits)
    ws = torch.empty(rows, dtype=torch.float32, device=logits.device)
    _lib.call("vit_softmax_xent", _ptr(logits), _ptr(labels), rows, classes, _ptr(loss), _ptr(dlogits), _ptr(ws),
              _stream(stream))
    return loss, dlogits


def adamw(table_dev, nchunks, lr, beta1, beta2, eps, weight_decay, bias_corr1, bias_corr2, grad_scale,
          shadow_dtype, stream=None):
    _lib.call("vit_adamw", _ptr(table_dev), nchunks, lr, beta1, beta2, eps, weight_decay, bias_corr1, bias_corr2,
              grad_scale, dtype_code(shadow_dtype), _stream(stream))


def pack(table_dev, nchunks, shadow_dtype, stream=None):
    _lib.call("vit_pack", _ptr(table_dev), nchunks, dtype_code(shadow_dtype), _stream(stream))


# elements per multi-tensor chunk (one 256-thread workgroup each).  Measured on the C2 parameter set
# (tools/adamw_bench.py, profiles/r60_adamw_chunk.log): 64 Ki 527 us, 16 Ki 476, 8 Ki 471, 4 Ki 473 — more, smaller
# workgroups keep more loads in flight per CU.  VIT_ADAMW_CHUNK overrides it.
CHUNK = int(os.environ.get("VIT_ADAMW_CHUNK", 8192))


def build_chunk_table(entries, device):
    """entries: list of (p, g, m, v, shadow) tensors (fp32 contiguous, shadow may be None).  Returns (uint8 device
    tensor holding the vit_tensor_chunk array, nchunks)."""
    chunks = []
    for p, g, m, v, sh in entries:
        n = p.numel()
        es = sh.element_size() if sh is not None else 0
        for off in range(0, n, CHUNK):
            c = _lib.TensorChunk()
            c.p = p.data_ptr() + 4 * off
            c.g = (g.data_ptr() + 4 * off) if g is not None else 0
            c.m = (m.data_ptr() + 4 * off) if m is not None else 0
            c.v = (v.data_ptr() + 4 * off) if v is not None else 0
            c.shadow = (sh.data_ptr() + es * off) if sh is not None else None
            c.n = min(CHUNK, n - off)
            chunks.append(c)
    arr = (_lib.TensorChunk * len(chunks))(*chunks)
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.to(device), len(chunks)
