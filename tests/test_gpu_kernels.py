"""Per-kernel numerics on the MI355X: each HIP kernel (called through the C-ABI) against a plain torch fp32/fp64
reference of the same op.  Integer-valued operands make the MFMA layout checks exact (asymmetric data, so a
transposed fragment or C-write cannot pass)."""
import math

import pytest
import torch

from oracle import vit_oracle as O

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from VisionTransformer import _lib, _ops  # noqa: E402

DEV = "cuda"


def _ints(shape, lo=-4, hi=5, gen=None, dtype=torch.bfloat16):
    return torch.randint(lo, hi, shape, generator=gen).to(dtype).to(DEV)


def _ref_op(A, B, akc, bkc):
    """C[i][j] = sum_r A(i,r) B(j,r) in float64 from the stored layouts."""
    Ai = A.double() if akc else A.double().t()
    Bj = B.double() if bkc else B.double().t()
    return Ai @ Bj.t()


LAYOUTS = [(True, True), (True, False), (False, False)]


@pytest.mark.parametrize("akc,bkc", LAYOUTS)
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 192), (200, 136, 72), (56, 40, 24), (136, 8, 2000)])
def test_gemm_bf16_exact_integers(akc, bkc, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = _ints((M, K) if akc else (K, M), gen=g)
    B = _ints((N, K) if bkc else (K, N), gen=g)
    C = torch.empty(M, N, dtype=torch.float32, device=DEV)
    _ops.gemm(A, B, C, M, N, K, A.stride(0), B.stride(0), N, a_kcontig=akc, b_kcontig=bkc)
    ref = _ref_op(A, B, akc, bkc)
    assert torch.equal(C.double(), ref), (C.double() - ref).abs().max()


@pytest.mark.parametrize("impl", ["2", "4"])
@pytest.mark.parametrize("akc,bkc", LAYOUTS)
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (520, 264, 640), (1000, 776, 128), (72, 520, 192),
                                   (2048, 768, 768)])
def test_gemm_bf16_kernels_exact(libopt, impl, akc, bkc, M, N, K):
    """Every LDS-DMA kernel variant (option gemm_impl) on ragged M/N tails and 1..12 k-tiles, exact on integers."""
    libopt("gemm_impl", int(impl))
    g = torch.Generator().manual_seed(M + 5 * N + 11 * K)
    A = _ints((M, K) if akc else (K, M), gen=g)
    B = _ints((N, K) if bkc else (K, N), gen=g)
    C = torch.empty(M, N, dtype=torch.float32, device=DEV)
    _ops.gemm(A, B, C, M, N, K, A.stride(0), B.stride(0), N, a_kcontig=akc, b_kcontig=bkc)
    ref = _ref_op(A, B, akc, bkc)
    assert torch.equal(C.double(), ref), (C.double() - ref).abs().max()
    Cb = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)      # bf16 output path of the same kernel
    _ops.gemm(A, B, Cb, M, N, K, A.stride(0), B.stride(0), N, a_kcontig=akc, b_kcontig=bkc)
    assert torch.equal(Cb, ref.float().bfloat16())


@pytest.mark.parametrize("impl", ["2", "4"])
@pytest.mark.parametrize("split", [3, 7])
def test_gemm_bf16_kernels_split_k(libopt, impl, split):
    """wgrad form with split-K (incl. an empty last slice: 10 k-tiles over 7 slices) on each kernel variant."""
    libopt("gemm_impl", int(impl))
    g = torch.Generator().manual_seed(split)
    M, N, K = 264, 776, 640
    A = _ints((K, M), gen=g)
    B = _ints((K, N), gen=g)
    C = _ints((M, N), gen=g, dtype=torch.float32)
    ref = C.double() * 1.0 + _ref_op(A, B, False, False)
    ws = torch.empty(split * M * N, dtype=torch.float32, device=DEV)
    _ops.gemm(A, B, C, M, N, K, M, N, N, a_kcontig=False, b_kcontig=False, beta=1.0, split_k=split, workspace=ws)
    assert torch.equal(C.double(), ref), (C.double() - ref).abs().max()


@pytest.mark.parametrize("variant", ["plain", "bias_relu", "bias_gelu", "aux", "bias_drop_res", "drop_res_f32",
                                     "alpha"])
def test_gemm_epilogue_kinds_match_general(libopt, variant):
    """The specialised v4 epilogues are bitwise equal to the general one (option gemm_epi_general)."""
    torch.manual_seed(7)
    M, N, K = 1000, 776, 256
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    bias = torch.randn(N, device=DEV)
    aux = torch.randn(M, N, device=DEV).bfloat16()
    res32 = torch.randn(M, N, device=DEV)
    kw = {"plain": {}, "bias_relu": dict(bias=bias, act=_ops.ACT_RELU), "bias_gelu": dict(bias=bias, act=_ops.ACT_GELU),
          "aux": dict(aux=aux, ldaux=N), "bias_drop_res": dict(bias=bias, dropout_p=0.2, seed=99, res=aux, ldres=N),
          "drop_res_f32": dict(dropout_p=0.3, seed=5, res=res32, ldres=N), "alpha": dict(alpha=0.37)}[variant]
    outs = []
    for general in ("0", "1"):
        libopt("gemm_epi_general", int(general))
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        _ops.gemm(x, w, out, M, N, K, K, K, N, **kw)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


def test_gemm_bf16_rejects_unaligned_contiguous_dim():
    A = torch.zeros(24, 50, dtype=torch.bfloat16, device=DEV)   # rowstrided A with M = 50 (not a multiple of 8)
    B = torch.zeros(24, 40, dtype=torch.bfloat16, device=DEV)
    C = torch.empty(50, 40, device=DEV)
    with pytest.raises(RuntimeError, match="multiple"):
        _ops.gemm(A, B, C, 50, 40, 24, 50, 40, 40, a_kcontig=False, b_kcontig=False)


@pytest.mark.parametrize("akc,bkc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(64, 64, 16), (100, 70, 33), (257, 130, 300), (10, 1000, 3072)])
def test_gemm_f32(akc, bkc, M, N, K):
    g = torch.Generator().manual_seed(1)
    A = torch.randn((M, K) if akc else (K, M), generator=g).to(DEV)
    B = torch.randn((N, K) if bkc else (K, N), generator=g).to(DEV)
    C = torch.empty(M, N, dtype=torch.float32, device=DEV)
    _ops.gemm(A, B, C, M, N, K, A.stride(0), B.stride(0), N, a_kcontig=akc, b_kcontig=bkc)
    ref = _ref_op(A, B, akc, bkc)
    tol = 2e-6 * math.sqrt(K) * ref.abs().max().item()
    assert (C.double() - ref).abs().max().item() <= tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogue_bias_relu_dropout_residual(dtype):
    torch.manual_seed(0)
    M, N, K = 394, 256, 128
    x = torch.randn(M, K, device=DEV).to(dtype)
    w = (torch.randn(N, K, device=DEV) * 0.1).to(dtype)
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV).to(dtype)
    out = torch.empty(M, N, dtype=dtype, device=DEV)
    seed, p = 1234, 0.2
    _ops.gemm(x, w, out, M, N, K, K, K, N, bias=bias, res=res, ldres=N, dropout_p=p, seed=seed)
    import numpy as np
    from oracle.vit_oracle import dropout_keep
    keep = dropout_keep(seed, (M, N), p).to(DEV)
    y = x.float() @ w.float().t() + bias
    ref = res.float() + y * keep * (1 / (1 - p))
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    assert (out.float() - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item())
    # relu + aux mask variants
    out2 = torch.empty(M, N, dtype=dtype, device=DEV)
    _ops.gemm(x, w, out2, M, N, K, K, K, N, bias=bias, act=_ops.ACT_RELU)
    ref2 = torch.relu(y)
    assert (out2.float() - ref2).abs().max().item() <= tol * max(1.0, ref2.abs().max().item())
    out3 = torch.empty(M, N, dtype=dtype, device=DEV)
    _ops.gemm(x, w, out3, M, N, K, K, K, N, aux=res, ldaux=N)
    ref3 = (x.float() @ w.float().t()) * (res.float() > 0)
    assert (out3.float() - ref3).abs().max().item() <= tol * max(1.0, ref3.abs().max().item())


@pytest.mark.parametrize("B,D", [(3, 256), (5, 768)])
def test_gemm_row_group_and_rowmod(libopt, B, D):
    """patch-embed epilogue: rows (b, n) -> b*T + n, + pos[n] (res_rowmod = N); the dedicated wide kind (EPI_PATCH)
    equals the general epilogue bit for bit and leaves the CLS rows alone"""
    torch.manual_seed(1)
    N, T, K = 196, 197, 768
    cols = torch.randn(B * N, K, device=DEV).bfloat16()
    w = (torch.randn(D, K, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(D, device=DEV)
    pos = torch.randn(T, D, device=DEV)
    outs = []
    for general in ("0", "1"):
        libopt("gemm_epi_general", int(general))
        x0 = torch.full((B * T, D), 7.0, device=DEV).bfloat16()
        _ops.gemm(cols, w, x0, B * N, D, K, K, K, D, bias=bias, res=pos, ldres=D, res_rowmod=N, out_group=(N, T))
        outs.append(x0)
    ref = (cols.float() @ w.float().t() + bias).view(B, N, D) + pos[:N]
    got = outs[0].view(B, T, D)
    assert (got[:, :N].float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    assert torch.all(got[:, N] == 7.0)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_split_k_wgrad(dtype):
    torch.manual_seed(2)
    M, N, K = 5000, 256, 192          # wgrad form: dW[N][K] = dY^T X with reduction over M rows
    dy = torch.randn(M, N, device=DEV).to(dtype)
    x = torch.randn(M, K, device=DEV).to(dtype)
    dw = torch.randn(N, K, device=DEV)
    dw0 = dw.clone()
    _ops.gemm(dy, x, dw, N, K, M, N, K, K, a_kcontig=False, b_kcontig=False, beta=1.0, split_k=7)
    ref = dw0.double() + dy.double().t() @ x.double()
    tol = (1e-5 if dtype == torch.float32 else 1e-5) * ref.abs().max().item() * 10
    assert (dw.double() - ref).abs().max().item() <= tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols", [64, 192, 768, 3072])
def test_layernorm_fwd_bwd(dtype, cols):
    torch.manual_seed(3)
    rows = 300
    x = (torch.randn(rows, cols, device=DEV) * 2 + 0.5).to(dtype)
    g = torch.rand(cols, device=DEV) + 0.5
    b = torch.randn(cols, device=DEV)
    y, mean, rstd = _ops.layernorm_fwd(x, g, b)
    xr = x.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (cols,), gr, br, 1e-5)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert (y.float() - yr).abs().max().item() <= tol * 4
    dy = torch.randn(rows, cols, device=DEV).to(dtype)
    dres = torch.randn(rows, cols, device=DEV).to(dtype)
    yr.backward(dy.float())
    dx = torch.empty_like(x)
    drop = torch.empty_like(x)
    part = _ops.layernorm_bwd(dy, x, g, mean, rstd, dx, dres=dres, drop_out=drop, drop_p=0.2, drop_seed=99,
                              osum=True)
    dg = torch.empty(cols, device=DEV)
    db = torch.empty(cols, device=DEV)
    _ops.colsum(part[0], part.shape[1], cols, cols, dg)
    ds = torch.full((cols,), 0.5, device=DEV)
    _ops.colsum_finish(part[1:], [db, ds])
    # third partial set: column sums of drop_out / (1 - p) — drop_out is stored unscaled (an exact mask), and the
    # sums are the bias gradient of the Linear it feeds
    ref_ds = drop.double().sum(0) * 1.25
    assert ((ds.double() - ref_ds).abs() <= 1e-5 * drop.double().abs().sum(0) + 1e-6).all()
    # without drop_out the third set sums dx_out
    dx2 = torch.empty_like(x)
    part2 = _ops.layernorm_bwd(dy, x, g, mean, rstd, dx2, dres=dres, osum=True)
    assert torch.equal(dx2, dx)
    s3 = [torch.zeros(cols, device=DEV) for _ in range(3)]
    _ops.colsum_finish(part2, s3)
    assert ((s3[2].double() - dx.double().sum(0)).abs() <= 1e-5 * dx.double().abs().sum(0) + 1e-6).all()
    assert torch.allclose(s3[0], dg, rtol=1e-5, atol=1e-5)
    ref_dx = xr.grad + dres.float()
    scale = ref_dx.abs().max().item()
    assert (dx.float() - ref_dx).abs().max().item() <= tol * 4 * scale
    assert (dg - gr.grad).abs().max().item() <= tol * 4 * gr.grad.abs().max().item()
    assert (db - br.grad).abs().max().item() <= tol * 4 * br.grad.abs().max().item()
    from oracle.vit_oracle import dropout_keep
    keep = dropout_keep(99, (rows, cols)).to(DEV)
    assert torch.equal(drop.float(), dx.float() * keep)


@pytest.mark.parametrize("dtype,cols", [(torch.bfloat16, 768), (torch.bfloat16, 1024), (torch.bfloat16, 3072),
                                        (torch.float32, 768), (torch.float32, 3072)])
def test_layernorm_bwd_many_rows_and_saved_mask(dtype, cols):
    """vit_layernorm_bwd at >= 8192 rows (every wave of a block busy, the next 4-row group prefetched, the per-wave LDS
    accumulators summed in wave order across many row groups; the fp32 NV 6-12 path included) against torch, and the
    saved-mask form (drop_mask: the forward's keep bits as a mask4, here packed from the same counter hash) bitwise
    equal to the hash form, dx, drop_out and every partial column sum alike."""
    from oracle.vit_oracle import dropout_keep
    torch.manual_seed(cols)
    rows = 8192 + 36
    x = (torch.randn(rows, cols, device=DEV) * 2 + 0.5).to(dtype)
    g = torch.rand(cols, device=DEV) + 0.5
    b = torch.randn(cols, device=DEV)
    y, mean, rstd = _ops.layernorm_fwd(x, g, b)
    dy = torch.randn(rows, cols, device=DEV).to(dtype)
    dres = torch.randn(rows, cols, device=DEV).to(dtype)
    xr = x.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xr, (cols,), gr, br, 1e-5).backward(dy.float())
    dx, drop = torch.empty_like(x), torch.empty_like(x)
    part = _ops.layernorm_bwd(dy, x, g, mean, rstd, dx, dres=dres, drop_out=drop, drop_p=0.2, drop_seed=7, osum=True)
    keep = dropout_keep(7, (rows, cols)).to(DEV)
    mask = _mask4_pack(keep.bool())
    dx2, drop2 = torch.empty_like(x), torch.empty_like(x)
    part2 = _ops.layernorm_bwd(dy, x, g, mean, rstd, dx2, dres=dres, drop_out=drop2, drop_p=0.2, drop_seed=7,
                               osum=True, drop_mask=mask)
    assert torch.equal(dx, dx2) and torch.equal(drop, drop2) and torch.equal(part, part2)
    assert torch.equal(drop.float(), dx.float() * keep)
    dg, db, ds = (torch.empty(cols, device=DEV) for _ in range(3))
    _ops.colsum_finish(part, [dg, db, ds])
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    ref_dx = xr.grad + dres.float()
    assert (dx.float() - ref_dx).abs().max().item() <= tol * 4 * ref_dx.abs().max().item()
    assert (dg - gr.grad).abs().max().item() <= tol * 4 * gr.grad.abs().max().item()
    assert (db - br.grad).abs().max().item() <= tol * 4 * br.grad.abs().max().item()
    ref_ds = drop.double().sum(0) * 1.25
    assert ((ds.double() - ref_ds).abs() <= 1e-5 * drop.double().abs().sum(0) + 1e-6).all()


@pytest.mark.parametrize("variant", ["plain", "aux", "bias_relu", "bias_drop_res", "f32_out", "v2_small"])
def test_gemm_colsum_part(variant):
    """Column sums of C as stored, fused into the v4 row epilogue (a separate pass for the other kernels / general
    epilogue), finished by vit_colsum_finish: the bias gradient of the Linear whose input gradient C is."""
    torch.manual_seed(11)
    M, N, K = (300, 200, 128) if variant == "v2_small" else (1000, 776, 256)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    bias = torch.randn(N, device=DEV)
    aux = torch.randn(M, N, device=DEV).bfloat16()
    out = torch.empty(M, N, dtype=torch.float32 if variant == "f32_out" else torch.bfloat16, device=DEV)
    part = torch.empty(_ops.colsum_part_rows(M), N, device=DEV)
    if variant == "aux":                                  # dgrad layout: B row-strided [K][N], ReLU-backward mask
        wt = w.t().contiguous()
        _ops.gemm(x, wt, out, M, N, K, K, N, N, b_kcontig=False, aux=aux, ldaux=N, colsum_part=part)
    else:
        kw = {"bias_relu": dict(bias=bias, act=_ops.ACT_RELU),
              "bias_drop_res": dict(bias=bias, dropout_p=0.2, seed=3, res=aux, ldres=N)}.get(variant, {})
        _ops.gemm(x, w, out, M, N, K, K, K, N, colsum_part=part, **kw)
    got = torch.full((N,), 0.5, device=DEV)
    _ops.colsum_finish(part, [got], beta=1.0)
    ref = out.double().sum(0) + 0.5
    assert ((got.double() - ref).abs() <= 1e-5 * out.double().abs().sum(0) + 1e-5).all()


@pytest.mark.parametrize("variant", ["plain", "bias_relu", "aux", "bias_drop_res"])
def test_gemm_split_k_tail(libopt, variant):
    """A v4 GEMM whose 256x256 tiles leave the last round of the 256 CUs at most half full runs the remaining tile
    rows split-K (M = 23140, N = 768, K = 2304: 91 x 3 tiles = 85 tile rows in whole rounds + 6 tile rows split 8 ways).
    Integer data: outputs and fused column sums equal the unsplit kernel's bit for bit, dropout masks included."""
    import ctypes
    from VisionTransformer import _lib
    g = torch.Generator().manual_seed(5)
    M, N, K = 90 * 256 + 100, 768, 2304
    libopt("gemm_tail", 1)                          # off by default since round 5 (the two-stream schedule)
    libopt("gemm_tail_min_kt", 32)                  # K = 2304 (36 k-tiles) is below the shipped minimum (40)
    d = _lib.GemmDesc()
    d.m, d.n, d.k, d.a_kcontig, d.b_kcontig, d.in_dtype, d.out_dtype = M, N, K, 1, 1, 1, 1
    assert _lib.load().vit_gemm_workspace_bytes(ctypes.byref(d)) == 8 * (M - 85 * 256) * N * 4
    a = _ints((M, K), gen=g)
    b = _ints((N, K), gen=g)
    bias = _ints((N,), gen=g, dtype=torch.float32)
    aux = _ints((M, N), gen=g)
    outs, parts = [], []
    for tail in ("0", "1"):
        libopt("gemm_tail", int(tail))
        c = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        p = torch.empty(_ops.colsum_part_rows(M), N, device=DEV)
        if variant == "aux":
            _ops.gemm(a, b.t().contiguous(), c, M, N, K, K, N, N, b_kcontig=False, aux=aux, ldaux=N, colsum_part=p)
        else:
            kw = {"bias_relu": dict(bias=bias, act=_ops.ACT_RELU),
                  "bias_drop_res": dict(bias=bias, dropout_p=0.2, seed=9, res=aux, ldres=N)}.get(variant, {})
            _ops.gemm(a, b, c, M, N, K, K, K, N, colsum_part=p, **kw)
        outs.append(c)
        parts.append(p)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(parts[0], parts[1])
    if variant == "plain":
        assert torch.equal(outs[1], (a.double() @ b.double().t()).float().bfloat16())


def _mask4_pack(bits):
    """bool [m, n] -> the VIT_MASK4 byte layout of include/vit_hip.h (byte ((i/4)*ceil(n/4) + j/4)*4 + i%4, bit j%4)."""
    m, n = bits.shape
    m4, n4 = -(-m // 4) * 4, -(-n // 4) * 4
    b = torch.zeros(m4, n4, dtype=torch.int32, device=bits.device)
    b[:m, :n] = bits.int()
    b = b.view(m4 // 4, 4, n4 // 4, 4).permute(0, 2, 1, 3)
    w = torch.tensor([1, 2, 4, 8], dtype=torch.int32, device=bits.device)
    return (b * w).sum(-1).to(torch.uint8).reshape(-1)


@pytest.mark.parametrize("variant", ["plain", "bias_relu", "bias_drop_res", "general", "tail", "f32_out", "ragged"])
def test_gemm_mask4_produce_consume(libopt, variant):
    """mask_out = C's mask4 (C as stored > 0; dropout keep bits when the epilogue drops out), and a mask4 aux masks the
    dgrad GEMM exactly as the bf16 tensor it was taken from (ReLU backward, transformer.py:57)."""
    torch.manual_seed(13)
    M, N, K = {"tail": (90 * 256 + 100, 768, 2304), "ragged": (1001, 776, 264)}.get(variant, (1000, 776, 256))
    if variant == "general":
        libopt("gemm_epi_general", 1)
    if variant == "tail":
        libopt("gemm_tail", 1)
        libopt("gemm_tail_min_kt", 32)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV).bfloat16()
    kw = {"bias_drop_res": dict(bias=bias, dropout_p=0.2, seed=3, res=res, ldres=N)}.get(
        variant, dict(bias=bias, act=_ops.ACT_RELU) if variant != "plain" else {})
    out = torch.empty(M, N, dtype=torch.float32 if variant == "f32_out" else torch.bfloat16, device=DEV)
    mask = torch.full((_ops.mask4_bytes(M, N),), 0xAA, dtype=torch.uint8, device=DEV)
    _ops.gemm(x, w, out, M, N, K, K, K, N, mask_out=mask, **kw)
    if variant == "bias_drop_res":
        from oracle.vit_oracle import dropout_keep
        want = dropout_keep(3, (M, N), 0.2).to(DEV) > 0
    else:
        want = out > 0
    # bytes of rows >= M (padding of the last 4-row group) are unspecified
    nq = -(-N // 4)
    b = torch.arange(mask.numel(), device=DEV)
    valid = (b // 4 // nq) * 4 + b % 4 < M
    assert torch.equal(mask[valid], _mask4_pack(want)[valid])
    # consumer: dgrad layout (B row-strided), mask4 aux == bf16 aux
    if variant in ("plain", "bias_drop_res", "f32_out"):
        return
    g = torch.randn(M, K, device=DEV).bfloat16()
    wt = (torch.randn(K, N, device=DEV) * 0.1).bfloat16()
    d_ref = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    d_m = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    p_ref = torch.empty(_ops.colsum_part_rows(M), N, device=DEV)
    p_m = torch.empty_like(p_ref)
    _ops.gemm(g, wt, d_ref, M, N, K, K, N, N, b_kcontig=False, aux=out, ldaux=N, colsum_part=p_ref, alpha=1.25)
    _ops.gemm(g, wt, d_m, M, N, K, K, N, N, b_kcontig=False, aux=mask, colsum_part=p_m, alpha=1.25)
    assert torch.equal(d_m, d_ref)
    assert torch.equal(p_m, p_ref)


@pytest.mark.parametrize("variant", ["plain", "plain_cs", "bias_relu_mask", "aux_cs", "auxm_cs", "bias_drop_res_mask",
                                     "grouped"])
def test_gemm_persistent_matches_one_per_item(libopt, variant):
    """The wide-epilogue kinds run on a persistent grid (one workgroup per CU looping over its tiles, the next tile's
    first stages staged during the current tile's epilogue).  With more tiles than CUs (ragged last tile row), outputs,
    masks and fused column sums equal the one-workgroup-per-tile launch (option gemm_persist 0) bit for bit; integer
    data makes the plain product exact."""
    g = torch.Generator().manual_seed(17)
    M, N, K = (4200, 4096, 192) if variant == "grouped" else (23 * 256 + 100, 3072, 256)   # 272 / 288 tiles
    a = _ints((M, K), gen=g)
    b = _ints((N, K), gen=g)
    bias = _ints((N,), gen=g, dtype=torch.float32)
    aux = _ints((M, N), gen=g)
    res = _ints((M, N), gen=g)
    mask_in = torch.randint(0, 256, (_ops.mask4_bytes(M, N),), generator=g, dtype=torch.uint8).to(DEV)
    results = []
    for persist in ("1", "0", "shared"):      # "shared": VIT_FLAG_SHARED_CUS (the data-parallel backward's launches)
        libopt("gemm_persist", 0 if persist == "0" else 1)
        sh = dict(shared_cus=persist == "shared")
        c = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        part = torch.empty(_ops.colsum_part_rows(M), N, device=DEV)
        mask = torch.full((_ops.mask4_bytes(M, N),), 0xAA, dtype=torch.uint8, device=DEV)
        if variant in ("aux_cs", "auxm_cs"):             # dgrad layout (B row-strided), ReLU-backward mask
            bt = b.t().contiguous()
            kw = dict(aux=aux, ldaux=N) if variant == "aux_cs" else dict(aux=mask_in)
            _ops.gemm(a, bt, c, M, N, K, K, N, N, b_kcontig=False, colsum_part=part, alpha=0.5, **kw, **sh)
        else:
            kw = {"plain_cs": dict(colsum_part=part), "bias_relu_mask": dict(bias=bias, act=_ops.ACT_RELU, mask_out=mask),
                  "bias_drop_res_mask": dict(bias=bias, dropout_p=0.2, seed=5, res=res, ldres=N, mask_out=mask)}.get(
                      variant, {})
            _ops.gemm(a, b, c, M, N, K, K, K, N, **kw, **sh)
        results.append((c, part if "cs" in variant else None, mask if "mask" in variant else None))
    (c1, p1, m1) = results[0]
    for c0, p0, m0 in results[1:]:
        assert torch.equal(c1, c0)
        if p1 is not None:
            assert torch.equal(p1, p0)
        if m1 is not None:
            assert torch.equal(m1, m0)
    if variant in ("plain", "grouped"):
        assert torch.equal(c1, (a.double() @ b.double().t()).float().bfloat16())


def _attn_flash_grads(qkv, d_o, B, T, H, hd, scale):
    """dQ|dK|dV [B*T, 3D] in fp64 between the bf16 storage points of the MFMA flash kernels (oracle
    _FlashBF16Attention: unnormalised P rounded to bf16 for P V, P rounded for dV = P^T dO, dS rounded for dQ / dK,
    delta = rowsum(dO * O) from the unrounded O) — the same-rounding reference for the bf16 kernel gates."""
    D = H * hd
    q, k, v = (t.detach().clone().requires_grad_(True)
               for t in qkv.double().view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4))
    o = O._FlashBF16Attention.apply(q, k, v, scale)
    o.backward(d_o.double().view(B, T, H, hd).transpose(1, 2))
    return torch.cat([t.grad.transpose(1, 2).reshape(B * T, D) for t in (q, k, v)], 1)


def _check_attn_bwd_bf16(dqkv, ref, D, tol=2e-2):
    """Norm-wise error of each of dQ, dK, dV against the same-rounding reference (relative to the larger of its own
    norm and 1e-3 of the whole gradient's)."""
    errs = {}
    floor = 1e-3 * float(ref.norm())            # T = 1: dQ = dK = 0 exactly (one key), the kernels leave ~1e-6
    for name, sl in (("dQ", slice(0, D)), ("dK", slice(D, 2 * D)), ("dV", slice(2 * D, 3 * D))):
        a, r = dqkv[:, sl].double(), ref[:, sl]
        errs[name] = float((a - r).norm() / max(float(r.norm()), floor, 1e-30))
    print("attention backward vs same-rounding fp64:", {k: f"{v:.2e}" for k, v in errs.items()})
    assert all(e <= tol for e in errs.values()), errs


def _attn_ref(qkv, B, T, H, hd, scale):
    D = H * hd
    q, k, v = qkv.float().view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * scale
    p = torch.softmax(s, -1)
    o = (p @ v).permute(0, 2, 1, 3).reshape(B * T, D)
    lse = torch.logsumexp(s, -1)
    return o, lse, p


@pytest.mark.parametrize("shape", ["proj_fwd", "fc2_fwd", "dgrad_qkv", "fc1_fwd", "dgrad_fc2m", "dgrad_proj"])
def test_gemm_c2_shapes_tail_split(libopt, shape):
    """The forward / input-gradient GEMMs at their real C2 shapes (M = 50,432: 591 / 2,364 tiles over 256 CUs, the
    persistent grid).  With the tails of a last partial round — the split-K tail (option gemm_tail: N = 768 and
    K >= 2048 run it split over K with fp32 slabs) and the 128x128-tile tail (option gemm_tail_v2: the K = 768 shapes
    run its tile rows as quarter tiles, two workgroups per CU; round 5) — against whole 256x256 tiles only: the same
    outputs to bf16 rounding of a different fp32 summation order, identical keep / ReLU bits where the pre-rounding
    values agree, bitwise run to run, and within bf16 tolerance of an fp32 torch product."""
    M, D = 256 * 197, 768
    libopt("gemm_tail", 1)                          # off by default since round 5 (the two-stream schedule)
    libopt("gemm_tail_min_kt", 32)                  # the QKV input gradient's tail too (K = 2304: 36 k-tiles)
    m, n, k, bkc, kind = {"proj_fwd": (M, D, D, True, "bdr"), "fc2_fwd": (M, D, 4 * D, True, "bdr"),
                          "dgrad_qkv": (M, D, 3 * D, False, "plain"), "fc1_fwd": (M, 4 * D, D, True, "relu_mask"),
                          "dgrad_fc2m": (M, 4 * D, D, False, "auxm"), "dgrad_proj": (M, D, D, False, "plain")}[shape]
    g = torch.Generator(device=DEV).manual_seed(11)
    a = (torch.rand(m, k, device=DEV, generator=g) * 2 - 1).bfloat16()
    b = (torch.rand(n, k, device=DEV, generator=g) * 2 - 1).bfloat16() if bkc else \
        (torch.rand(k, n, device=DEV, generator=g) * 2 - 1).bfloat16()
    bias = torch.randn(n, device=DEV, generator=g)
    res = torch.randn(m, n, device=DEV, generator=g).bfloat16()
    mask_in = torch.randint(0, 256, (_ops.mask4_bytes(m, n),), device=DEV, generator=g, dtype=torch.uint8)
    ws = torch.empty(64 << 20, dtype=torch.float32, device=DEV)

    def run():
        c = torch.empty(m, n, dtype=torch.bfloat16, device=DEV)
        mask = torch.zeros(_ops.mask4_bytes(m, n), dtype=torch.uint8, device=DEV)
        kw = {"bdr": dict(bias=bias, dropout_p=0.2, seed=3, res=res, ldres=n, mask_out=mask),
              "relu_mask": dict(bias=bias, act=_ops.ACT_RELU, mask_out=mask), "auxm": dict(aux=mask_in),
              "plain": {}}[kind]
        _ops.gemm(a, b, c, m, n, k, k, k if bkc else n, n, b_kcontig=bkc, workspace=ws, **kw)
        return c, mask

    c1, m1 = run()
    c1b, m1b = run()
    assert torch.equal(c1, c1b) and torch.equal(m1, m1b)                 # deterministic
    libopt("gemm_tail", 0)
    libopt("gemm_tail_v2", 0)
    c0, m0 = run()
    ref = a.float() @ (b.float().t() if bkc else b.float())
    scale = float(ref.abs().max())
    d = (c1.float() - c0.float()).abs()
    assert float(d.max()) <= 2 ** -7 * max(scale, 1.0), float(d.max())    # summation order only (bf16 ulps)
    assert float((d > 0).float().mean()) < 0.02
    if kind == "plain":
        assert float((c1.float() - ref).abs().max()) <= 2 ** -7 * scale
    if kind in ("bdr", "relu_mask"):
        assert float((m1 != m0).float().mean()) < 1e-3                 # bits flip only where a value sits at 0


@pytest.mark.parametrize("dtype,hd", [(torch.float32, 16), (torch.float32, 64), (torch.bfloat16, 64),
                                      (torch.bfloat16, 32)])
@pytest.mark.parametrize("T", [5, 17, 197, 577])
@pytest.mark.parametrize("amp", [0.15, 1.0])
def test_attention_fwd_bwd(dtype, hd, T, amp):
    torch.manual_seed(T + hd)
    B, H = 2, 3
    D = H * hd
    scale = hd ** 0.5                     # the reference multiplies by sqrt(hd) (transformer.py:24)
    qkv = (torch.randn(B * T, 3 * D, device=DEV) * amp).to(dtype)
    o, lse = _ops.attn_fwd(qkv, B, T, H, hd, scale)
    x = qkv.float().requires_grad_(True)
    o_ref, lse_ref, _ = _attn_ref(x, B, T, H, hd, scale)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert (o.float() - o_ref).abs().max().item() <= tol * max(1.0, o_ref.abs().max().item())
    assert (lse - lse_ref).abs().max().item() <= 1e-3 * max(1.0, lse_ref.abs().max().item())
    d_o = torch.randn(B * T, D, device=DEV).to(dtype)
    if dtype == torch.float32:
        dqkv = _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, scale)
        o_ref.backward(d_o.float())
        g = x.grad
        err = (dqkv.float() - g).abs().max().item()
        assert err <= tol * 5 * max(1.0, g.abs().max().item()), err
        return
    # bf16: against an fp64 evaluation between the kernels' own bf16 storage points, 2e-2 of the
    # norm of each of dQ / dK / dV (was 10% of the max); the engine's path (exact delta: o32 where the tiled T > 256
    # backward takes it)
    o32 = torch.empty(B * T, D, device=DEV) if _ops.attn_bwd_uses_o32(B, T, H, hd, dtype) else None
    if o32 is not None:
        o2, lse2 = _ops.attn_fwd(qkv, B, T, H, hd, scale, o32=o32)
        assert torch.equal(o2, o) and torch.equal(lse2, lse)
    dqkv = _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, scale, o32=o32)
    _check_attn_bwd_bf16(dqkv, _attn_flash_grads(qkv, d_o, B, T, H, hd, scale), D)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("T,hd", [(1, 64), (5, 64), (197, 64), (197, 32), (577, 64), (2500, 16), (65, 128), (197, 20)])
def test_attention_row0_fwd_bwd(dtype, T, hd):
    """Query 0 only (vit_attn_fwd_row0 / vit_attn_bwd_row0, the pruned last block; hd = 20: the generic one-key-per-
    thread kernels, the rest the lane-chunk kernels): o row 0 and lse[.., 0] equal the
    full attention's row 0; with an output gradient on row 0 only, dQ row 0 and all of dK / dV equal the full
    backward's, and the dQ rows 1..T-1 (and o rows 1..T-1) are left untouched.  fp32 to 2e-5 of the largest value
    (1e-4 for dQ0) against fp64, bf16 to 1e-2 of the norm (the kernels compute in fp32 and round once)."""
    torch.manual_seed(T + hd)
    B, H = 3, 2
    D = H * hd
    scale = hd ** 0.5
    qkv = (torch.randn(B * T, 3 * D, device=DEV) * 0.5).to(dtype)
    o = torch.full((B * T, D), 7.0, device=DEV, dtype=dtype)
    o, lse = _ops.attn_fwd_row0(qkv, B, T, H, hd, scale, o=o)
    x = qkv.double().requires_grad_(True)
    q, k, v = x.view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * scale
    p = torch.softmax(s, -1)
    o_ref = (p @ v).permute(0, 2, 1, 3).reshape(B * T, D)
    rows = torch.arange(B, device=DEV) * T
    others = torch.ones(B * T, dtype=torch.bool, device=DEV)
    others[rows] = False
    assert bool((o[others] == 7.0).all())                               # untouched
    got, ref = o[rows].double(), o_ref[rows].detach()
    if dtype == torch.float32:
        assert float((got - ref).abs().max()) <= 2e-5 * max(1.0, float(ref.abs().max()))
    else:
        assert float((got - ref).norm() / ref.norm()) < 1e-2
    lse_ref = torch.logsumexp(s, -1)[:, :, 0]
    assert float((lse[:, :, 0].double() - lse_ref).abs().max()) <= 1e-4 * max(1.0, float(lse_ref.abs().max()))
    g0 = torch.randn(B, D, device=DEV).to(dtype)
    d_o = torch.zeros(B * T, D, device=DEV, dtype=torch.float64)
    d_o[rows] = g0.double()
    o_ref.backward(d_o)
    dqkv = torch.full((B * T, 3 * D), 5.0, device=DEV, dtype=dtype)
    dqkv[:, D:] = 0
    _ops.attn_bwd_row0(qkv, g0, D, dqkv, B, T, H, hd, scale)
    torch.cuda.synchronize()
    assert bool((dqkv[others, :D] == 5.0).all())                       # dQ rows 1..T-1 untouched
    gref = x.grad
    floor = 1e-3 * float(gref.abs().max())       # T = 1: dQ0 is 0 exactly (one key), the kernel's is rounding-sized
    for name, sel in (("dQ0", (rows, slice(0, D))), ("dK", (slice(None), slice(D, 2 * D))),
                      ("dV", (slice(None), slice(2 * D, 3 * D)))):
        a, r = dqkv[sel].double(), gref[sel]
        if dtype == torch.float32:
            # dQ0 = scale sum_k dS_k K_k with sum_k dS_k = 0: a cancelling sum, gated at the fp32 parity bound (1e-4)
            err = float((a - r).abs().max()) / max(floor, float(r.abs().max()))
            assert err <= (1e-4 if name == "dQ0" else 2e-5), (name, err)
        else:
            err = float((a - r).norm() / max(float(r.norm()), floor * r.numel() ** 0.5))
            assert err < 1e-2, (name, err)
    again = torch.full_like(dqkv, 5.0)
    again[:, D:] = 0
    _ops.attn_bwd_row0(qkv, g0, D, again, B, T, H, hd, scale)
    assert torch.equal(again, dqkv)                                     # deterministic


@pytest.mark.parametrize("B,H,T", [(1, 1, 1), (3, 3, 33), (3, 3, 65), (1, 5, 129), (3, 1, 300), (2, 3, 577)])
def test_attention_tiled_kernels_any_grid(libopt, B, H, T):
    """The tiled T > 256 kernels forced at any T (attn_fwd_split / attn_bwd_split): the XCD-aware (block, head) remap
    over grids of nblk x B*H workgroups that are not multiples of 8, LDS-DMA tiles whose rows >= T are clamped to row
    T - 1 (masked), the skipped all-padding sub-blocks and delta formed in the dQ kernel — against fp32 torch."""
    torch.manual_seed(T + 7 * H)
    hd = 64
    D = H * hd
    scale = 8.0
    qkv = (torch.randn(B * T, 3 * D, device=DEV) * 0.5).bfloat16()
    libopt("attn_fwd_split", 1)
    libopt("attn_bwd_split", 1)
    o, lse = _ops.attn_fwd(qkv, B, T, H, hd, scale)
    x = qkv.float().requires_grad_(True)
    o_ref, lse_ref, _ = _attn_ref(x, B, T, H, hd, scale)
    assert (o.float() - o_ref).abs().max().item() <= 2e-2 * max(1.0, o_ref.abs().max().item())
    assert (lse - lse_ref).abs().max().item() <= 1e-3 * max(1.0, lse_ref.abs().max().item())
    d_o = torch.randn(B * T, D, device=DEV).bfloat16()
    o32 = torch.empty(B * T, D, device=DEV)             # exact delta, as the engine runs the tiled backward
    o2, _ = _ops.attn_fwd(qkv, B, T, H, hd, scale, o32=o32)
    assert torch.equal(o2, o)
    dqkv = _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, scale, o32=o32)
    _check_attn_bwd_bf16(dqkv, _attn_flash_grads(qkv, d_o, B, T, H, hd, scale), D)
    again = _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, scale, o32=o32)
    assert torch.equal(again, dqkv)                    # deterministic


@pytest.mark.parametrize("T", [1, 31, 32, 33, 197, 256])
def test_attention_bwd_fused_matches_split(libopt, T):
    """The one-workgroup-per-(image, head) backward (T <= 256) against the split dQ / dK-dV kernels and fp64."""
    torch.manual_seed(T)
    B, H, hd = 2, 3, 64
    D = H * hd
    qkv = (torch.randn(B * T, 3 * D, device=DEV) * 0.5).bfloat16()
    o, lse = _ops.attn_fwd(qkv, B, T, H, hd, 8.0)
    d_o = torch.randn(B * T, D, device=DEV).bfloat16()
    fused = _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, 8.0)
    libopt("attn_bwd_split", 1)
    split = _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, 8.0)
    x = qkv.double().requires_grad_(True)
    q, k, v = x.view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
    p = torch.softmax((q @ k.transpose(-1, -2)) * 8.0, -1)
    (p @ v).permute(0, 2, 1, 3).reshape(B * T, D).backward(d_o.double())
    g = x.grad
    ef = (fused.double() - g).abs().max().item()
    es = (split.double() - g).abs().max().item()
    assert ef <= max(2 * es, 1e-2 * max(1.0, g.abs().max().item())), (ef, es)
    assert (fused.float() - split.float()).abs().max().item() <= 2e-2 * max(1.0, g.abs().max().item())


@pytest.mark.parametrize("grid", [0, 7, 100])
def test_attention_bwd_shared_cus_bitwise(libopt, grid):
    """VIT_FLAG_SHARED_CUS (one workgroup per (image, head) instead of the persistent grid that stages the next item
    during the current one) and persistent grids of other sizes (attn_bwd_grid; 0 = one per CU): bitwise the same
    dQ / dK / dV, with more items than workgroups (the in-kernel delta is a fixed-order sum)."""
    torch.manual_seed(3)
    B, H, hd, T = 24, 12, 64, 197                       # 288 items
    D = H * hd
    qkv = (torch.randn(B * T, 3 * D, device=DEV) * 0.5).bfloat16()
    o, lse = _ops.attn_fwd(qkv, B, T, H, hd, 8.0)
    d_o = torch.randn(B * T, D, device=DEV).bfloat16()
    b = _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, 8.0, shared_cus=True)    # one workgroup per item
    libopt("attn_bwd_grid", grid)
    a = _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, 8.0)
    assert torch.equal(a, b)


@pytest.mark.parametrize("T", [197, 209, 240, 256])
def test_attention_fwd_ring_ragged_grids(libopt, T):
    """The persistent ring forward (attn_fwd_ring<NT>) where workgroups take several items and the item count is not a
    multiple of the grid: B = 17, H = 12 (204 items) over 64 and 192 workgroups (per call, max_wgs)
    and over the option attn_fwd_grid; T = 197 is the 3-slot ring (NT 13), T = 209 / 240 / 256 the 2-slot ring (NT
    14-16).  Against fp64 on the same bf16 inputs (o to 2e-2 of the largest value, lse to 1e-3), bitwise equal over
    every grid (items are independent), and within the same gate of the one-workgroup-per-item forward."""
    torch.manual_seed(T)
    B, H, hd = 17, 12, 64
    D = H * hd
    qkv = (torch.randn(B * T, 3 * D, device=DEV) * 0.5).bfloat16()
    x = qkv.double()
    q, k, v = x.view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * 8.0
    o_ref = (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(B * T, D)
    lse_ref = torch.logsumexp(s, -1)
    scale_o = max(1.0, float(o_ref.abs().max()))
    outs = []
    for wgs, opt in ((64, 0), (192, 0), (0, 0), (0, 50)):
        libopt("attn_fwd_grid", opt)
        o = torch.full((B * T, D), 3.0, device=DEV, dtype=torch.bfloat16)
        lse = torch.full((B, H, T), 3.0, device=DEV)
        o, lse = _ops.attn_fwd(qkv, B, T, H, hd, 8.0, o=o, lse=lse, max_wgs=wgs)
        torch.cuda.synchronize()
        err = float((o.double() - o_ref).abs().max())
        assert err <= 2e-2 * scale_o, (wgs, opt, err)
        assert float((lse.double() - lse_ref).abs().max()) <= 1e-3 * max(1.0, float(lse_ref.abs().max())), (wgs, opt)
        outs.append((o, lse))
    for o, lse in outs[1:]:
        assert torch.equal(o, outs[0][0]) and torch.equal(lse, outs[0][1])
    libopt("attn_fwd_grid", 0)
    libopt("attn_fwd_ring", 0)
    of, lf = _ops.attn_fwd(qkv, B, T, H, hd, 8.0)
    assert float((of.double() - outs[0][0].double()).abs().max()) <= 2e-2 * scale_o
    assert float((lf - outs[0][1]).abs().max()) <= 1e-3 * max(1.0, float(lse_ref.abs().max()))


@pytest.mark.parametrize("T", [1, 31, 32, 33, 197, 256])
def test_attention_fwd_fused_matches_split(libopt, T):
    """The one-workgroup-per-(image, head) forward (T <= 256) against the 128-query-tile kernel and fp32."""
    torch.manual_seed(T + 1)
    B, H, hd = 2, 3, 64
    qkv = (torch.randn(B * T, 3 * H * hd, device=DEV) * 0.5).bfloat16()
    of, lf = _ops.attn_fwd(qkv, B, T, H, hd, 8.0)
    libopt("attn_fwd_split", 1)
    osp, lsp = _ops.attn_fwd(qkv, B, T, H, hd, 8.0)
    o_ref, lse_ref, _ = _attn_ref(qkv, B, T, H, hd, 8.0)
    ef = (of.float() - o_ref).abs().max().item()
    es = (osp.float() - o_ref).abs().max().item()
    assert ef <= max(2 * es, 1e-2 * max(1.0, o_ref.abs().max().item())), (ef, es)
    assert (lf - lse_ref).abs().max().item() <= 1e-3 * max(1.0, lse_ref.abs().max().item())
    assert (lf - lsp).abs().max().item() <= 1e-3 * max(1.0, lsp.abs().max().item())


def test_attention_probs_generic():
    torch.manual_seed(5)
    B, T, H, hd = 2, 17, 2, 64
    qkv = (torch.randn(B * T, 3 * H * hd, device=DEV) * 0.2)
    probs = torch.empty(B, H, T, T, device=DEV)
    _ops.attn_fwd(qkv, B, T, H, hd, hd ** 0.5, probs=probs)
    _, _, p = _attn_ref(qkv, B, T, H, hd, hd ** 0.5)
    assert (probs - p).abs().max().item() < 1e-5


def test_colsum_finish_batch_matches_single():
    """vit_colsum_finish_batch (one launch for an encoder block's bias / LN-affine gradient sums) gives each job's
    outputs bitwise as its own vit_colsum_finish, beta included."""
    g = torch.Generator(device=DEV).manual_seed(5)
    jobs = [(197, 3072, 1, 0.0), (1576, 768, 3, 1.0), (1576, 768, 2, 0.5), (3, 100, 1, 0.0)]
    parts = [torch.randn(ns, nparts, cols, device=DEV, generator=g) for nparts, cols, ns, _ in jobs]
    init = [[torch.randn(cols, device=DEV, generator=g) for _ in range(ns)] for _, cols, ns, _ in jobs]
    single = [[t.clone() for t in outs] for outs in init]
    for p, outs, (_, _, _, beta) in zip(parts, single, jobs):
        _ops.colsum_finish(p, outs, beta=beta)
    batch = [[t.clone() for t in outs] for outs in init]
    _ops.colsum_finish_batch([(p, outs, beta) for p, outs, (_, _, _, beta) in zip(parts, batch, jobs)])
    for a, b in zip(single, batch):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    assert torch.allclose(single[0][0], parts[0][0].double().sum(0).float(), rtol=1e-5, atol=1e-4)


def test_misc_kernels():
    torch.manual_seed(6)
    # im2col (vit.py:21-29 conv as GEMM)
    x = torch.randn(2, 3, 64, 48, device=DEV)
    cols = _ops.im2col(x, 16, torch.float32)
    ref = x.view(2, 3, 4, 16, 3, 16).permute(0, 2, 4, 1, 3, 5).reshape(2 * 12, 768)
    assert torch.equal(cols, ref)
    colsb = _ops.im2col(x, 16, torch.bfloat16)
    assert torch.equal(colsb, ref.bfloat16())
    # colsum
    a = torch.randn(1000, 300, device=DEV)
    out = torch.ones(300, device=DEV)
    _ops.colsum(a, 1000, 300, 300, out, beta=1.0)
    assert (out - (a.sum(0) + 1)).abs().max().item() < 1e-3
    # copy2d with grouped source rows + accumulate
    src = torch.randn(4 * 5, 8, device=DEV)
    dst = torch.ones(4 * 3, 8, device=DEV)
    _ops.copy2d(src, 8, dst, 8, 12, 8, group=(3, 5), beta=1.0)
    assert torch.allclose(dst, src.view(4, 5, 8)[:, :3].reshape(12, 8) + 1)
    # the 16-B raw path (same dtype, no beta, aligned): bit-exact, grouped rows (the patch-gradient gather), strided
    # rows, and an unaligned leading dimension that must take the element path
    for dt in (torch.bfloat16, torch.float32):
        src = torch.randn(6 * 197, 776, device=DEV).to(dt)
        dst = torch.zeros(6 * 196, 768, device=DEV, dtype=dt)
        _ops.copy2d(src, 776, dst, 768, 6 * 196, 768, group=(196, 197))
        assert torch.equal(dst, src.view(6, 197, 776)[:, :196, :768].reshape(6 * 196, 768))
        d2 = torch.zeros(6, 768 + 4, device=DEV, dtype=dt)
        _ops.copy2d(src, 197 * 776, d2, 768 + 4, 6, 768)
        assert torch.equal(d2[:, :768], src.view(6, 197, 776)[:, 0, :768]) and bool((d2[:, 768:] == 0).all())
        d3 = torch.zeros(5, 12, device=DEV, dtype=dt)
        _ops.copy2d(src, 3, d3, 12, 5, 12)
        assert torch.equal(d3, torch.as_strided(src, (5, 12), (3, 1)))
    # GELU
    z = torch.randn(5000, device=DEV) * 3
    assert (_ops.gelu_fwd(z) - torch.nn.functional.gelu(z)).abs().max().item() < 1e-5
    zr = z.clone().requires_grad_(True)
    torch.nn.functional.gelu(zr).backward(torch.ones_like(z))
    assert (_ops.gelu_bwd(z, torch.ones_like(z)) - zr.grad).abs().max().item() < 1e-5
    # softmax cross entropy (train.py:81,93)
    lg = torch.randn(37, 1000, device=DEV) * 4
    lb = torch.randint(0, 1000, (37,), device=DEV)
    loss, dl = _ops.softmax_xent(lg, lb)
    lr_ = lg.clone().requires_grad_(True)
    lref = torch.nn.functional.cross_entropy(lr_, lb)
    lref.backward()
    assert abs(loss.item() - lref.item()) < 1e-5
    assert (dl - lr_.grad).abs().max().item() < 1e-6
    # dropout backward mask
    from oracle.vit_oracle import dropout_keep
    t = torch.randn(3000, device=DEV)
    y = torch.empty_like(t)
    _ops.dropout_bwd(t, y, 0.2, 4242)
    keep = dropout_keep(4242, (3000,)).to(DEV)
    assert torch.equal(y, t * keep * 1.25)


def test_adamw_matches_torch():
    torch.manual_seed(7)
    shapes = [(300,), (70000,), (128, 64)]
    ps = [torch.randn(s, device=DEV) for s in shapes]
    gs = [torch.randn(s, device=DEV) for s in shapes]
    ms = [torch.zeros_like(p) for p in ps]
    vs = [torch.zeros_like(p) for p in ps]
    sh = [torch.empty(s, dtype=torch.bfloat16, device=DEV) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt = torch.optim.AdamW(ref, lr=1e-3, weight_decay=1e-4)
    table, n = _ops.build_chunk_table(list(zip(ps, gs, ms, vs, sh)), DEV)
    for step in range(1, 4):
        for r, g in zip(ref, gs):
            r.grad = g.clone()
        opt.step()
        _ops.adamw(table, n, 1e-3, 0.9, 0.999, 1e-8, 1e-4, 1 - 0.9 ** step, 1 - 0.999 ** step, 1.0, torch.bfloat16)
    for p, r, s in zip(ps, ref, sh):
        assert (p - r.detach()).abs().max().item() < 1e-6
        assert torch.equal(s, p.bfloat16())
