"""FusedAdamW step time on the ViT-B/16 parameter set (91.4 M fp32 parameters in 562 tensors, bf16 shadows).

    python tools/adamw_bench.py [--reps 30]        (VIT_HIP_LIB=... for a variant library)

Prints the mean of the HIP-event-timed steps and the rate over the 30 B per parameter the step must move (read p, g,
m, v; write p, m, v and the bf16 shadow)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    from VisionTransformer import config, vit
    from VisionTransformer.optim import FusedAdamW, cross_entropy
    dev = torch.device("cuda", 0)
    cfg = config.ViTConfig.preset("base", img_size=224, batch_size=8, num_classes=1000, precision=torch.bfloat16,
                                  device="cpu")
    torch.manual_seed(0)
    model = vit.VisionTransformer(cfg).to(dev).train()
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    x = torch.randn(8, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (8,), device=dev)
    cross_entropy(model(x), y).backward()          # real gradients in the flat buffer
    for _ in range(3):
        opt.step()
    torch.cuda.synchronize()
    n = sum(p.numel() for p in model.parameters())
    ts = []
    for _ in range(args.reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        opt.step()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    med = ts[len(ts) // 2]
    print(f"FusedAdamW step, {n / 1e6:.1f} M params: median {med * 1e3:.1f} us, "
          f"{30 * n / (med * 1e-3) / 1e12:.2f} TB/s (30 B/param)", flush=True)


if __name__ == "__main__":
    main()
