"""Time LayerNorm fwd/bwd and the fused-column-sum finish at the ViT-B/16 B=256 shape (50432 x 768 bf16).
    python tools/ln_bench.py [--reps 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
import torch  # noqa: E402
from VisionTransformer import _ops  # noqa: E402


def timeit(fn, reps):
    ts = []
    for i in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    rows, cols = 256 * 197, 768
    torch.manual_seed(0)
    x = torch.randn(rows, cols, device="cuda").bfloat16()
    g, b = torch.rand(cols, device="cuda") + 0.5, torch.randn(cols, device="cuda")
    dy, dres = torch.randn_like(x), torch.randn_like(x)
    y, mean, rstd = _ops.layernorm_fwd(x, g, b)
    dx, drop = torch.empty_like(x), torch.empty_like(x)
    part = _ops.layernorm_bwd(dy, x, g, mean, rstd, dx, dres=dres, drop_out=drop, drop_p=0.2, drop_seed=1, osum=True)
    outs = [torch.empty(cols, device="cuda") for _ in range(3)]
    t = timeit(lambda: _ops.layernorm_fwd(x, g, b, y=y), args.reps)
    print(f"ln fwd              {t:7.1f} us  {2 * rows * cols * 2 / t / 1e6:6.2f} TB/s")
    t = timeit(lambda: _ops.layernorm_bwd(dy, x, g, mean, rstd, dx, dres=dres, drop_out=drop, drop_p=0.2,
                                          drop_seed=1, partial=part, osum=True), args.reps)
    print(f"ln bwd (+osum)      {t:7.1f} us  {5 * rows * cols * 2 / t / 1e6:6.2f} TB/s")
    mask = torch.randint(0, 256, (_ops.mask4_bytes(rows, cols),), dtype=torch.uint8, device="cuda")
    t = timeit(lambda: _ops.layernorm_bwd(dy, x, g, mean, rstd, dx, dres=dres, drop_out=drop, drop_p=0.2,
                                          drop_mask=mask, partial=part, osum=True), args.reps)
    print(f"ln bwd (+osum,mask) {t:7.1f} us  {5 * rows * cols * 2 / t / 1e6:6.2f} TB/s")
    t = timeit(lambda: _ops.layernorm_bwd(dy, x, g, mean, rstd, dx, dres=dres, partial=part, osum=True), args.reps)
    print(f"ln bwd (no drop)    {t:7.1f} us  {4 * rows * cols * 2 / t / 1e6:6.2f} TB/s")
    t = timeit(lambda: _ops.colsum_finish(part, outs), args.reps)
    print(f"colsum_finish x3    {t:7.1f} us")


if __name__ == "__main__":
    main()
