"""Time the attention kernels at the ViT-B/16 training shape (B=256, T=197, H=12, hd=64, bf16).
    python tools/attn_bench.py [--reps 20]"""
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--T", type=int, default=197, help="tokens (577 = 384^2 / patch 16 + cls: the tiled kernels)")
    args = ap.parse_args()
    B, T, H, hd = args.batch, args.T, 12, 64
    D = H * hd
    torch.manual_seed(0)
    qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).bfloat16()
    o, lse = _ops.attn_fwd(qkv, B, T, H, hd, 8.0)
    d_o = torch.randn(B * T, D, device="cuda").bfloat16()
    fl_f = 4.0 * B * H * T * T * hd
    fl_b = 10.0 * B * H * T * T * hd
    t = timeit(lambda: _ops.attn_fwd(qkv, B, T, H, hd, 8.0), args.reps)
    print(f"attn fwd          {t:8.1f} us  {fl_f / t / 1e6:7.1f} TF (4 T^2 hd per head)")
    t = timeit(lambda: _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, 8.0), args.reps)
    print(f"attn bwd fused    {t:8.1f} us  {fl_b / t / 1e6:7.1f} TF (10 T^2 hd per head)")
    # the training configuration: the forward also stores O in fp32, the backward forms delta from it (attn_delta)
    o32 = torch.empty(B * T, D, device="cuda")
    t = timeit(lambda: _ops.attn_fwd(qkv, B, T, H, hd, 8.0, o32=o32), args.reps)
    print(f"attn fwd +o32     {t:8.1f} us  {fl_f / t / 1e6:7.1f} TF")
    t = timeit(lambda: _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, 8.0, o32=o32), args.reps)
    print(f"attn bwd +delta   {t:8.1f} us  {fl_b / t / 1e6:7.1f} TF (attn_delta from o32 + fused)")
    os.environ["VIT_ATTN_BWD_SPLIT"] = "1"
    t = timeit(lambda: _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, 8.0), args.reps)
    print(f"attn bwd split    {t:8.1f} us  {fl_b / t / 1e6:7.1f} TF")
    os.environ.pop("VIT_ATTN_BWD_SPLIT")


if __name__ == "__main__":
    main()
