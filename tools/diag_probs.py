"""Diagnostic: per-layer max |P_ours - P_fp64| of the attention probabilities (tiny config, depth 12)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from oracle import vit_oracle as O  # noqa: E402
from VisionTransformer import config, vit  # noqa: E402

torch.set_num_threads(16)
cfg = O.make_config("tiny", img=64, batch=8)
st = O.init_state(cfg, 0)
x, y = O.synthetic_batch(cfg)
with torch.no_grad():
    _, p64 = O.forward(st, x, cfg, dtype=torch.float64, keep_probs=True)
    _, p32 = O.forward(st, x, cfg, keep_probs=True)
c = config.ViTConfig(3, 10, cfg.num_patches, cfg.embedding_size, 16, cfg.num_heads, 12, "cpu", 8)
m = vit.VisionTransformer(c)
m.load_state_dict(st)
m = m.cuda().eval()
m.store_attention_probs = True
with torch.no_grad():
    m(x.cuda())
for l in range(12):
    po = m.transformer_encoder.blocks[l].multi_head.attention_probs.cpu().double()
    d_o = (po - p64[l]).abs()
    d_3 = (p32[l].double() - p64[l]).abs()
    idx = torch.nonzero(d_o == d_o.max())[0].tolist()
    print(f"layer {l:2d}: ours max|dP| {d_o.max():.2e} at {idx}   oracle32 {d_3.max():.2e}")
