"""Interleaved A/B of libvit_hip.so builds on the ViT GEMM shapes (one process, rounds alternate between builds:
cdna_hip_programming.md §5.4 rule 24).  Each build is loaded RTLD_LOCAL, so several coexist.

    python tools/gemm_ab.py LIB1.so LIB2.so@VIT_GEMM_GROUP=4 ... [--reps 10] [--shapes fwd_qkv,...]

A build spec may carry `@NAME=VALUE[,NAME=VALUE]`: library options (vit_set_option) set around that build's calls,
e.g. `libvit_hip.so@gemm_tail=0`.  Prints the median time per (shape, build) and TF/s; checks outputs bitwise
against the first ("=" / "!"), and reports the largest relative difference to it."""  
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
import torch  # noqa: E402
from VisionTransformer import _lib  # noqa: E402  (GemmDesc layout)

M, D = 256 * 197, 768
SHAPES = {  # name: m, n, k, a_kcontig, b_kcontig, epilogue
    "fwd_qkv": (M, 3 * D, D, True, True, None), "fwd_proj": (M, D, D, True, True, "bdr"),
    "fwd_fc1": (M, 4 * D, D, True, True, "bias_relu"), "fwd_fc2": (M, D, 4 * D, True, True, "bdr"),
    "dgrad_fc2": (M, 4 * D, D, True, False, "aux"), "dgrad_fc2m": (M, 4 * D, D, True, False, "auxm"),
    "fwd_fc1m": (M, 4 * D, D, True, True, "bias_relu_m"), "dgrad_fc1": (M, D, 4 * D, True, False, None),
    "dgrad_qkv": (M, D, 3 * D, True, False, None), "dgrad_proj": (M, D, D, True, False, None),
    "wgrad_fc1": (4 * D, D, M, False, False, "wgrad"), "wgrad_fc2": (D, 4 * D, M, False, False, "wgrad"),
    "wgrad_qkv": (3 * D, D, M, False, False, "wgrad"), "wgrad_proj": (D, D, M, False, False, "wgrad"),
    "sq8192": (8192, 8192, 8192, True, True, None),
    # the input-gradient GEMMs with a transposed weight copy (B k-contiguous, the forward layout; round 6)
    "dgrad_fc2m_kc": (M, 4 * D, D, True, True, "auxm"), "dgrad_fc1_kc": (M, D, 4 * D, True, True, None),
    "dgrad_qkv_kc": (M, D, 3 * D, True, True, None), "dgrad_proj_kc": (M, D, D, True, True, None),
    # the proj / fc2 epilogue's parts (round 6): plain, bias + residual, + dropout, + dropout keep bits (the engine's)
    "fwd_proj_plain": (M, D, D, True, True, None), "fwd_proj_br": (M, D, D, True, True, "br"),
    "fwd_proj_bdrm": (M, D, D, True, True, "bdrm"), "fwd_fc2_plain": (M, D, 4 * D, True, True, None),
    "fwd_fc2_br": (M, D, 4 * D, True, True, "br"), "fwd_fc2_bdrm": (M, D, 4 * D, True, True, "bdrm"),
    # the same square GEMM in the dgrad (A k-contiguous, B row-strided) and weight-gradient (both row-strided, f32 out)
    # operand layouts: what the transposed LDS reads cost the k-loop
    "sq8192_kr": (8192, 8192, 8192, True, False, None), "sq8192_rr": (8192, 8192, 8192, False, False, "wgrad"),
    # one-round grids (epilogue cost vs how many CUs store at once)
    "fc1m_t24": (512, 4 * D, D, True, True, "bias_relu_m"), "fc1m_t96": (2048, 4 * D, D, True, True, "bias_relu_m"),
    "fc1m_t252": (5376, 4 * D, D, True, True, "bias_relu_m"), "fc1m_t504": (10752, 4 * D, D, True, True, "bias_relu_m"),
}


def load(path):
    lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL)
    lib.vit_gemm.argtypes = [ctypes.POINTER(_lib.GemmDesc), ctypes.c_void_p]
    lib.vit_gemm_workspace_bytes.argtypes = [ctypes.POINTER(_lib.GemmDesc)]
    lib.vit_gemm_workspace_bytes.restype = ctypes.c_int64
    lib.vit_gemm_split_k_hint.argtypes = [ctypes.c_int64] * 3 + [ctypes.c_int]
    lib.vit_last_error.restype = ctypes.c_char_p
    lib.vit_set_option.argtypes = [ctypes.c_char_p, ctypes.c_int64]
    lib.vit_get_option.argtypes = [ctypes.c_char_p]
    lib.vit_get_option.restype = ctypes.c_int64
    return lib


def desc(a, b, c, m, n, k, akc, bkc, epi, split, ws, aux, bias, res, mask):
    d = _lib.GemmDesc()
    d.a, d.b, d.c = a.data_ptr(), b.data_ptr(), c.data_ptr()
    d.lda, d.ldb, d.ldc = a.stride(0), b.stride(0), n
    d.m, d.n, d.k = m, n, k
    d.a_kcontig, d.b_kcontig = int(akc), int(bkc)
    d.in_dtype = _lib.BF16
    d.out_dtype = _lib.F32 if epi == "wgrad" else _lib.BF16
    d.alpha, d.beta = 1.0, 0.0
    if epi in ("bias_relu", "bias_relu_m", "bdr", "bdrm", "br"):
        d.bias = bias.data_ptr()
    if epi in ("bias_relu", "bias_relu_m"):
        d.act = _lib.ACT_RELU
    if epi == "bias_relu_m":
        d.mask_out = mask.data_ptr()
    if epi == "auxm":
        d.aux, d.ldaux, d.aux_dtype = mask.data_ptr(), 0, _lib.MASK4
    if epi == "aux":
        d.aux, d.ldaux, d.aux_dtype = aux.data_ptr(), n, _lib.BF16
    if epi in ("bdr", "bdrm", "br"):
        d.res, d.ldres, d.res_dtype = res.data_ptr(), n, _lib.BF16
    if epi in ("bdr", "bdrm"):
        d.dropout_p, d.dropout_seed = 0.2, 7
    if epi == "bdrm":
        d.mask_out = mask.data_ptr()
    d.split_k = split
    d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    specs = [(s.split("@")[0], dict(kv.split("=") for kv in s.split("@")[1].split(",")) if "@" in s else {})
             for s in args.libs]
    cache = {}
    libs = [None if p == "torch" else cache.setdefault(p, load(p)) for p, _ in specs]
    envs = [e for _, e in specs]
    names = ["torch" if p == "torch" else os.path.basename(p).replace("libvit_hip_", "").replace(".so", "") +
             ("@" + ",".join(f"{k}={v}" for k, v in e.items()) if e else "") for p, e in specs]
    ws = torch.empty(96 << 20, dtype=torch.float32, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(0)
    for sname in args.shapes.split(","):
        m, n, k, akc, bkc, epi = SHAPES[sname]
        a = (torch.rand((m, k) if akc else (k, m), device="cuda", generator=g) * 2 - 1).bfloat16()
        b = (torch.rand((n, k) if bkc else (k, n), device="cuda", generator=g) * 2 - 1).bfloat16()
        aux = (torch.rand(m, n, device="cuda", generator=g) - 0.3).bfloat16()
        res = torch.randn(m, n, device="cuda", generator=g).bfloat16()
        bias = torch.randn(n, device="cuda", generator=g)
        mask = torch.randint(0, 256, (4 * ((m + 3) // 4) * ((n + 3) // 4),), device="cuda", generator=g,
                             dtype=torch.uint8)
        c = torch.empty(m, n, dtype=torch.float32 if epi == "wgrad" else torch.bfloat16, device="cuda")
        split = next(l for l in libs if l is not None).vit_gemm_split_k_hint(m, n, k, _lib.BF16) if epi == "wgrad" else 1
        times = {nm: [] for nm in names}
        outs = {}
        for rep in range(args.reps + 2):
            for nm, lib, env in zip(names, libs, envs):
                saved = {kk: lib.vit_get_option(kk.encode()) for kk in env} if lib is not None else {}
                for kk, vv in env.items():
                    lib.vit_set_option(kk.encode(), int(vv))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if lib is None:   # "torch": hipBLASLt plain GEMM of the same operands (no epilogue), reference only
                    at = a if akc else a.t()
                    bt = b.t() if bkc else b
                    e0.record()
                    torch.mm(at, bt, out=c if c.dtype == torch.bfloat16 else None)
                    e1.record()
                    rc = 0
                else:
                    d = desc(a, b, c, m, n, k, akc, bkc, epi, split, ws, aux, bias, res, mask)
                    e0.record()
                    rc = lib.vit_gemm(ctypes.byref(d), stream)
                    e1.record()
                torch.cuda.synchronize()
                for kk, vv in saved.items():
                    lib.vit_set_option(kk.encode(), vv)
                if rc != 0:
                    sys.exit(f"{nm}: vit_gemm failed: {lib.vit_last_error().decode()}")
                if rep >= 2:
                    times[nm].append(e0.elapsed_time(e1) / 1e3)
                if rep == 2:
                    outs[nm] = c.clone()
        flop = 2.0 * m * n * k
        line = f"{sname:10s} split={split:2d}"
        for nm in names:
            t = sorted(times[nm])[len(times[nm]) // 2]
            same = "=" if torch.equal(outs[nm], outs[names[0]]) else \
                f"!{float((outs[nm].float() - outs[names[0]].float()).abs().max() / outs[names[0]].float().abs().max()):.0e}"
            if nm == "torch":
                same = "~"
            line += f" | {nm}: {t * 1e6:7.1f}us {flop / t / 1e12:7.1f}TF {same}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
