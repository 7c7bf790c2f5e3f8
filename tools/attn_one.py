"""Run the bf16 attention backward at the ViT-B/16 shape a few times (for rocprofv3 counters).
    python tools/attn_one.py [fused|split] [batch]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
mode = sys.argv[1] if len(sys.argv) > 1 else "fused"
if mode == "split":
    os.environ["VIT_ATTN_BWD_SPLIT"] = "1"
import torch  # noqa: E402
from VisionTransformer import _ops  # noqa: E402

B, T, H, hd = int(sys.argv[2]) if len(sys.argv) > 2 else 256, 197, 12, 64
D = H * hd
torch.manual_seed(0)
qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).bfloat16()
o, lse = _ops.attn_fwd(qkv, B, T, H, hd, 8.0)
d_o = torch.randn(B * T, D, device="cuda").bfloat16()
for _ in range(3):
    _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, 8.0)
torch.cuda.synchronize()
print("done")
