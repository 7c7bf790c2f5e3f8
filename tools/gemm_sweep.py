"""K sweep of the bf16 GEMM (fixed M, N): separates per-tile fixed cost from the per-k-tile main-loop cost.
    python tools/gemm_sweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
import torch  # noqa: E402
from VisionTransformer import _ops  # noqa: E402


def t_gemm(m, n, k, reps=10):
    a = (torch.rand(m, k, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(n, k, device="cuda") * 2 - 1).bfloat16()
    c = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
    ts = []
    for r in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _ops.gemm(a, b, c, m, n, k, k, k, n)
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1) / 1e3)
    return sorted(ts)[len(ts) // 2]


for m, n in ((50432, 3072), (50432, 768)):
    for k in (128, 256, 512, 768, 1536, 3072, 6144):
        t = t_gemm(m, n, k)
        print(f"m={m} n={n} k={k:5d}: {t*1e6:8.1f} us  {2*m*n*k/t/1e12:7.1f} TF", flush=True)
