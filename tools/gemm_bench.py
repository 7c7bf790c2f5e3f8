"""A/B the bf16 GEMM kernels on the ViT-B/16 (B=256) training shapes, interleaved in one process.
    python tools/gemm_bench.py [--impls 1,2] [--reps 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
import torch  # noqa: E402
from VisionTransformer import _lib, _ops  # noqa: E402

M, D = 256 * 197, 768
SHAPES = [  # name, m, n, k, a_kcontig, b_kcontig  (C = A(i,r) B(j,r))
    ("fwd qkv", M, 3 * D, D, True, True), ("fwd proj", M, D, D, True, True),
    ("fwd fc1", M, 4 * D, D, True, True), ("fwd fc2", M, D, 4 * D, True, True),
    ("dgrad fc2", M, 4 * D, D, True, False), ("dgrad fc1", M, D, 4 * D, True, False),
    ("dgrad qkv", M, D, 3 * D, True, False),
    ("wgrad fc1", 4 * D, D, M, False, False), ("wgrad fc2", D, 4 * D, M, False, False),
    ("wgrad qkv", 3 * D, D, M, False, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", default="4")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated shape names (default: all)")
    ap.add_argument("--no-ref", action="store_true", help="skip the hipBLASLt row")
    ap.add_argument("--epi", action="store_true", help="apply the engine's fused epilogue of each shape "
                    "(bias+ReLU, bias+dropout+residual, ReLU-backward mask)")
    args = ap.parse_args()
    impls = args.impls.split(",")
    torch.manual_seed(0)
    ws = torch.empty(64 << 20, dtype=torch.float32, device="cuda")
    only = [x.strip() for x in args.only.split(",") if x.strip()]
    for name, m, n, k, akc, bkc in SHAPES:
        if only and name not in only:
            continue
        a = (torch.rand((m, k) if akc else (k, m), device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand((n, k) if bkc else (k, n), device="cuda") * 2 - 1).bfloat16()
        wgrad = not akc
        c = torch.empty(m, n, dtype=torch.float32 if wgrad else torch.bfloat16, device="cuda")
        split = 1
        if wgrad:
            from VisionTransformer._engine import split_k_for
            split = split_k_for(m, n, k, torch.bfloat16)
        kw = {}
        if args.epi and not wgrad:
            bias = torch.randn(n, device="cuda")
            if name == "fwd fc1":
                kw = dict(bias=bias, act=_ops.ACT_RELU)
            elif name in ("fwd proj", "fwd fc2"):
                kw = dict(bias=bias, res=torch.randn(m, n, device="cuda").bfloat16(), ldres=n, dropout_p=0.2,
                          seed=7)
            elif name == "dgrad fc2":
                kw = dict(aux=torch.randn(m, n, device="cuda").bfloat16(), ldaux=n)
        res = {}
        outs = {}
        for rep in range(args.reps + 2):
            for impl in impls:
                _lib.set_option("gemm_impl", int(impl))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _ops.gemm(a, b, c, m, n, k, a.stride(0), b.stride(0), n, a_kcontig=akc, b_kcontig=bkc,
                          split_k=split, workspace=ws, **kw)
                e1.record()
                torch.cuda.synchronize()
                if rep >= 2:
                    res.setdefault(impl, []).append(e0.elapsed_time(e1) / 1e3)
                outs[impl] = c.float().clone() if rep == 2 else outs.get(impl)
        # hipBLASLt (torch.matmul) on the same operand layouts, plain GEMM without epilogue: a ceiling reference
        A = a if akc else a.t()
        Bm = b.t() if bkc else b
        tb = []
        for rep in range(0 if args.no_ref else args.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            torch.matmul(A, Bm)
            e1.record()
            torch.cuda.synchronize()
            if rep >= 2:
                tb.append(e0.elapsed_time(e1) / 1e3)
        flop = 2.0 * m * n * k
        line = f"{name:10s} m={m:6d} n={n:5d} k={k:6d} split={split:2d}"
        for impl in impls:
            t = sorted(res[impl])[len(res[impl]) // 2]
            line += f" | v{impl}: {t*1e6:8.1f}us {flop/t/1e12:7.1f} TF"
        if tb:
            tbl = sorted(tb)[len(tb) // 2]
            line += f" | hipBLASLt: {tbl*1e6:8.1f}us {flop/tbl/1e12:7.1f} TF"
        if len(impls) > 1:
            d = (outs[impls[0]] - outs[impls[1]]).abs().max().item()
            line += f" | maxdiff {d:.3g}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
