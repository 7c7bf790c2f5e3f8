"""Time vit_adamw on the ViT-B/16 parameter set (C2: 562 tensors, 86.6M fp32 elements + bf16 shadows) for several
multi-tensor chunk sizes (elements per workgroup).  usage: python tools/adamw_bench.py [--reps 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vision-transformer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from VisionTransformer import _ops, config, vit
    dev = torch.device("cuda", 0)
    cfg = config.ViTConfig.preset("base", img_size=224, batch_size=256, num_classes=1000, device="cpu")
    m = vit.VisionTransformer(cfg).to(dev)
    ps = [p.detach() for p in m.parameters()]
    gs = [torch.randn_like(p) for p in ps]
    ms = [torch.zeros_like(p) for p in ps]
    vs = [torch.zeros_like(p) for p in ps]
    sh = [torch.empty(p.shape, dtype=torch.bfloat16, device=dev) for p in ps]
    n = sum(p.numel() for p in ps)
    for chunk in (65536, 32768, 16384, 8192, 4096):
        _ops.CHUNK = chunk
        tab, nc = _ops.build_chunk_table(list(zip(ps, gs, ms, vs, sh)), dev)
        ts = []
        for i in range(args.reps + 3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _ops.adamw(tab, nc, 1e-4, 0.9, 0.999, 1e-8, 1e-4, 0.1, 0.001, 1.0, torch.bfloat16)
            e1.record()
            torch.cuda.synchronize()
            if i >= 3:
                ts.append(e0.elapsed_time(e1) * 1e3)
        t = sorted(ts)[len(ts) // 2]
        print(f"chunk {chunk:6d}: {nc:6d} workgroups, {t:7.1f} us, {n * 30 / t / 1e6:.2f} TB/s (30 B / element)")


if __name__ == "__main__":
    main()
