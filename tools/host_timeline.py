"""Host vs GPU timeline of the C2 training step (bench.py's step): where the host enqueues each phase and whether the GPU
had already drained its queue when the host got there (then the GPU idles on the host).

For each timed step: host milliseconds spent in model(x), cross_entropy, zero_grad, loss.backward and opt.step, and — via
an event recorded on the compute stream at each phase boundary and queried right away — whether the GPU had already
finished everything enqueued before that point ("drained"), plus the GPU time from step start to each boundary.
Steps run back to back as in bench.py (one synchronization at the end).
usage: python tools/host_timeline.py [--steps 10] [--engine ATTR=INT ...]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vision-transformer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--engine", action="append", default=[])
    args = ap.parse_args()
    from VisionTransformer import config, vit
    from VisionTransformer.optim import FusedAdamW, cross_entropy
    dev = torch.device("cuda", 0)
    cfg = config.ViTConfig.preset("base", img_size=224, batch_size=args.batch, num_classes=1000,
                                  precision=torch.bfloat16, device="cpu")
    torch.manual_seed(0)
    model = vit.VisionTransformer(cfg).to(dev).train()
    for kv in args.engine:
        k, v = kv.split("=")
        cur = getattr(model.hip_engine, k)
        setattr(model.hip_engine, k, bool(int(v)) if isinstance(cur, bool) else int(v))
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    x = torch.randn(args.batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (args.batch,), device=dev)
    names = ["forward", "xent", "zero_grad", "backward", "step"]
    rows = []
    for it in range(args.warmup + args.steps):
        s = torch.cuda.current_stream(dev)
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        evs, hs, drained = [], [], []
        t = time.perf_counter()
        for ph in names:
            if ph == "forward":
                logits = model(x)
            elif ph == "xent":
                loss = cross_entropy(logits, y)
            elif ph == "zero_grad":
                opt.zero_grad(set_to_none=True)
            elif ph == "backward":
                loss.backward()
            else:
                opt.step()
            t1 = time.perf_counter()
            hs.append((t1 - t) * 1e3)
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(dev))
            drained.append(e.query())
            evs.append(e)
            t = time.perf_counter()
        if it >= args.warmup:
            rows.append((hs, e0, evs, drained))
    torch.cuda.synchronize()
    rows = [(hs, [e0.elapsed_time(e) for e in evs], dr) for hs, e0, evs, dr in rows]
    print("| phase | host ms (mean) | GPU ms from step start to phase end (mean) | steps where the GPU had drained |")
    print("|---|---|---|---|")
    for i, ph in enumerate(names):
        h = sum(r[0][i] for r in rows) / len(rows)
        g = sum(r[1][i] for r in rows) / len(rows)
        d = sum(1 for r in rows if r[2][i])
        print(f"| {ph} | {h:.3f} | {g:.3f} | {d}/{len(rows)} |")
    print(f"\nhost total {sum(sum(r[0]) for r in rows) / len(rows):.3f} ms/step; GPU step "
          f"{sum(r[1][-1] for r in rows) / len(rows):.3f} ms (steps back to back, no synchronization: 'drained' = the "
          "host was behind the GPU at that phase boundary)")


if __name__ == "__main__":
    main()
