"""Time the attention kernels at the ViT-B/16 training shape (B=256, T=197, H=12, hd=64, bf16) and check the
backward against an fp64 torch evaluation on the same bf16 inputs (a few images).
    python tools/attn_bench.py [--reps 20] [--T 577]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
import torch  # noqa: E402
from VisionTransformer import _lib, _ops  # noqa: E402


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


def ref_grads(qkv, d_o, B, T, H, hd, scale, nb):
    """fp64 dQ/dK/dV of images 0..nb-1 (torch autograd on the bf16 values)."""
    D = H * hd
    x = qkv[:nb * T].double().view(nb, T, 3, H, hd).permute(2, 0, 3, 1, 4).detach().requires_grad_(True)
    q, k, v = x[0], x[1], x[2]
    p = torch.softmax(q @ k.transpose(-1, -2) * scale, dim=-1)
    o = p @ v
    g = d_o[:nb * T].double().view(nb, T, H, hd).permute(0, 2, 1, 3)
    (o * g).sum().backward()
    return x.grad.permute(1, 3, 0, 2, 4).reshape(nb * T, 3 * D)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--T", type=int, default=197, help="tokens (577 = 384^2 / patch 16 + cls: the tiled kernels)")
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--opt", action="append", default=[], help="library option name=value (A/B runs)")
    args = ap.parse_args()
    for kv in args.opt:
        name, val = kv.split("=")
        _lib.load().vit_set_option(name.encode(), int(val))
        print(f"option {name} = {val}")
    B, T, H, hd = args.batch, args.T, args.H, 64
    D = H * hd
    scale = 8.0
    torch.manual_seed(0)
    qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).bfloat16()
    o, lse = _ops.attn_fwd(qkv, B, T, H, hd, scale)
    d_o = torch.randn(B * T, D, device="cuda").bfloat16()
    fl_f = 4.0 * B * H * T * T * hd
    fl_b = 10.0 * B * H * T * T * hd
    uses_o32 = _ops.attn_bwd_uses_o32(B, T, H, hd, torch.bfloat16)
    o32 = torch.empty(B * T, D, device="cuda") if uses_o32 else None
    t = timeit(lambda: _ops.attn_fwd(qkv, B, T, H, hd, scale, o32=o32), args.reps)
    print(f"attn fwd (training form{', +o32' if uses_o32 else ''})  {t:8.1f} us  {fl_f / t / 1e6:7.1f} TF "
          f"(4 T^2 hd per head)")
    ws = torch.empty(_ops.attn_bwd_workspace_bytes(B, T, H, hd, torch.bfloat16) // 4 + 1, device="cuda")
    dq = torch.empty_like(qkv)
    t = timeit(lambda: _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, scale, dqkv=dq, workspace=ws, o32=o32), args.reps)
    print(f"attn bwd ({'tiled, delta in the dQ kernel' if uses_o32 else 'fused, in-kernel delta'})  {t:8.1f} us  "
          f"{fl_b / t / 1e6:7.1f} TF (10 T^2 hd per head)")
    nb = 4
    ref = ref_grads(qkv, d_o, B, T, H, hd, scale, nb)
    got = dq[:nb * T].double()
    for name, sl in (("dQ", slice(0, D)), ("dK", slice(D, 2 * D)), ("dV", slice(2 * D, 3 * D))):
        err = float((got[:, sl] - ref[:, sl]).norm() / ref[:, sl].norm())
        print(f"  {name} rel err vs fp64 (images 0..{nb - 1}): {err:.2e}")
    if not uses_o32:
        with _lib.option("attn_bwd_split", 1):
            o32s = torch.empty(B * T, D, device="cuda")
            _ops.attn_fwd(qkv, B, T, H, hd, scale, o32=o32s)
            t = timeit(lambda: _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, scale, dqkv=dq, workspace=ws, o32=o32s),
                       args.reps)
            print(f"attn bwd tiled (dq with delta from o32, dkdv)  {t:8.1f} us  {fl_b / t / 1e6:7.1f} TF")


if __name__ == "__main__":
    main()
