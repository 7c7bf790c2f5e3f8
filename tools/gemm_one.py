"""Run one bf16 GEMM shape a few times (for rocprofv3 counter collection).
    python tools/gemm_one.py M N K [impl] [layout]      layout: kk (default), kr (B row-strided), rr (both)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
import torch  # noqa: E402
from VisionTransformer import _ops  # noqa: E402

m, n, k = (int(v) for v in sys.argv[1:4])
if len(sys.argv) > 4 and sys.argv[4] != "0":
    os.environ["VIT_GEMM_IMPL"] = sys.argv[4]
lay = sys.argv[5] if len(sys.argv) > 5 else "kk"
akc, bkc = lay[0] == "k", lay[1] == "k"
a = (torch.rand((m, k) if akc else (k, m), device="cuda") * 2 - 1).bfloat16()
b = (torch.rand((n, k) if bkc else (k, n), device="cuda") * 2 - 1).bfloat16()
c = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
for _ in range(5):
    _ops.gemm(a, b, c, m, n, k, a.stride(0), b.stride(0), n, a_kcontig=akc, b_kcontig=bkc)
torch.cuda.synchronize()
print("done")
