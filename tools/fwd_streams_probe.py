"""Probe: the training forward of ViT-B/16 (B=256) in one stream vs two independent B=128 forwards on two streams at
once (what a two-micro-batch forward could gain from filling each other's idle CUs).  Timing only.
    python tools/fwd_streams_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
import torch  # noqa: E402
from VisionTransformer import config, vit  # noqa: E402


def make(b):
    cfg = config.ViTConfig.preset("base", img_size=224, batch_size=b, num_classes=1000, precision=torch.bfloat16,
                                  device="cpu")
    torch.manual_seed(0)
    m = vit.VisionTransformer(cfg).cuda().train()
    m.hip_engine.ensure_ready(torch.device("cuda", 0))
    return m


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    m256, ma, mb = make(256), make(128), make(128)
    x = torch.randn(256, 3, 224, 224, device="cuda")
    xa, xb = x[:128].contiguous(), x[128:].contiguous()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def one():
        return m256.hip_engine.forward(x, True, True)

    def two_serial():
        ma.hip_engine.forward(xa, True, True)
        mb.hip_engine.forward(xb, True, True)

    def two():
        sa.wait_stream(main_s)
        sb.wait_stream(main_s)
        with torch.cuda.stream(sa):
            ta = ma.hip_engine.forward(xa, True, True)
        with torch.cuda.stream(sb):
            tb = mb.hip_engine.forward(xb, True, True)
        main_s.wait_stream(sa)
        main_s.wait_stream(sb)
        return ta, tb

    for name, fn in (("B=256 one stream", one), ("2 x B=128 serial", two_serial), ("2 x B=128 two streams", two),
                     ("B=256 one stream", one), ("2 x B=128 two streams", two)):
        print(f"{name:24s} {timeit(fn):8.3f} ms", flush=True)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def step_probe():
    """Whole forward + backward (no optimizer): B=256 vs two B=128 models on two streams at once."""
    from VisionTransformer.optim import cross_entropy
    m256, ma, mb = make(256), make(128), make(128)
    x = torch.randn(256, 3, 224, 224, device="cuda")
    y = torch.randint(0, 1000, (256,), device="cuda")
    xa, xb, ya, yb = x[:128].contiguous(), x[128:].contiguous(), y[:128].contiguous(), y[128:].contiguous()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def fb(m, xx, yy):
        for p in m.parameters():
            p.grad = None
        cross_entropy(m(xx), yy).backward()

    def one():
        fb(m256, x, y)

    def two():
        sa.wait_stream(main_s)
        sb.wait_stream(main_s)
        with torch.cuda.stream(sa):
            fb(ma, xa, ya)
        with torch.cuda.stream(sb):
            fb(mb, xb, yb)
        main_s.wait_stream(sa)
        main_s.wait_stream(sb)

    for name, fn in (("fwd+bwd B=256", one), ("fwd+bwd 2 x B=128 streams", two), ("fwd+bwd B=256", one),
                     ("fwd+bwd 2 x B=128 streams", two)):
        print(f"{name:28s} {timeit(fn, 10):8.3f} ms", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "step":
    step_probe()
