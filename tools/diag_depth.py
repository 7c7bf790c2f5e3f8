"""Diagnostic: per-parameter gradient error vs fp64 oracle at several depths, for the HIP fp32 path and the CPU fp32
oracle.  python tools/diag_depth.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from oracle import vit_oracle as O  # noqa: E402
from VisionTransformer import config, vit  # noqa: E402

torch.set_num_threads(16)


def rel(a, b):
    return float((a.double() - b.double()).norm() / max(b.double().norm(), 1e-30))


for L in (1, 2, 4, 8, 12):
    cfg = O.make_config("tiny", img=64, batch=8, blocks=L)
    st = O.init_state(cfg, 0)
    x, y = O.synthetic_batch(cfg)
    _, _, g64 = O.loss_and_grads(st, x, y, cfg, dtype=torch.float64)
    _, _, g32 = O.loss_and_grads(st, x, y, cfg)
    c = config.ViTConfig(3, 10, cfg.num_patches, cfg.embedding_size, 16, cfg.num_heads, L, "cpu", 8)
    m = vit.VisionTransformer(c)
    m.load_state_dict(st)
    m = m.cuda().eval()
    lg = m(x.cuda())
    torch.nn.functional.cross_entropy(lg, y.cuda()).backward()
    rows = []
    for k, p in m.named_parameters():
        rows.append((rel(p.grad.cpu(), g64[k]), rel(g32[k], g64[k]), k))
    rows.sort(key=lambda r: -r[0] / max(r[1], 1e-12))
    print(f"L={L}: worst ratios (ours, oracle32):")
    for r in rows[:6]:
        print(f"   ours {r[0]:.2e}  oracle32 {r[1]:.2e}  {r[2]}")
    sys.stdout.flush()
