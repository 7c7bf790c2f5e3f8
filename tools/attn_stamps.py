"""Per-section cycles of the fused attention backward's steady iterations (diagnostic build with -DATT_STAMPS=1):
    VIT_HIP_LIB=tools/variants/libvit_hip_attstamps.so python tools/attn_stamps.py
Sections per iteration and wave: dq_store | back | front | dq | prefetch | barrier wait (to the next iteration)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
import torch  # noqa: E402
from VisionTransformer import _lib, _ops  # noqa: E402

B, T, H, hd = 256, 197, 12, 64
D = H * hd
torch.manual_seed(0)
qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).bfloat16()
o, lse = _ops.attn_fwd(qkv, B, T, H, hd, 8.0)
d_o = torch.randn(B * T, D, device="cuda").bfloat16()
ws = torch.empty(_ops.attn_bwd_workspace_bytes(B, T, H, hd, torch.bfloat16) // 4 + 1, device="cuda")
for _ in range(3):
    dq = _ops.attn_bwd(qkv, o, d_o, lse, B, T, H, hd, 8.0, workspace=ws)
torch.cuda.synchronize()
lib = _lib.load()
buf = (ctypes.c_ulonglong * (16 * 8 * 8 * 6))()
assert lib.vit_diag_attn_stamps(buf, 16 * 8 * 8 * 6) == 0
st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(16, 8, 8, 6)
names = ["dq_store", "back", "front", "dq", "prefetch", "barrier->next"]
rows = []
for wg in range(16):
    for w in range(8):
        for it in range(3, 6):           # iterations 3..6 of 7 (it+1 exists for the barrier span)
            s = st[wg, w, it]
            nxt = st[wg, w, it + 1, 0]
            if s[0] == 0 or nxt == 0:
                continue
            rows.append([s[1] - s[0], s[2] - s[1], s[3] - s[2], s[4] - s[3], s[5] - s[4], nxt - s[5]])
r = np.array(rows)
print(f"{len(r)} (workgroup, wave, iteration) samples; shader cycles (s_memtime)")
for i, n in enumerate(names):
    print(f"  {n:14s} median {np.median(r[:, i]):8.0f}  p90 {np.percentile(r[:, i], 90):8.0f}")
tot = r.sum(1)
print(f"  {'iteration':14s} median {np.median(tot):8.0f}")
# per wave (wave 7 has no key block)
for w in range(8):
    sel = [np.median([st[wg, w, it, 5] - st[wg, w, it, 0] for wg in range(16) if st[wg, w, it, 0]]) for it in (3, 4, 5)]
    print(f"  wave {w}: busy (stamp 0 -> 5) per iteration {np.median(sel):8.0f}")

# whole items: the first two items of workgroups 0-15
ib = (ctypes.c_ulonglong * (16 * 8 * 2 * 10))()
assert lib.vit_diag_attn_istamps(ib, 16 * 8 * 2 * 10) == 0
it_ = np.frombuffer(ib, dtype=np.uint64).astype(np.int64).reshape(16, 8, 2, 10)
labels = ["item wait (vmcnt(0) + sync)", "interval 0 (front 0)", "interval 1 (back 0, front 1)",
          "interval 2 (back 1, front 2, dq 0)", "steady iterations 3..nqb-1", "tail A (back last, dq)",
          "tail B (dq last)", "last dq_store", "K staging + dK/dV stores"]
print("whole items (median over workgroups, waves 0-6, both items), shader cycles:")
tot = 0
for k in range(9):
    d = it_[:, :7, :, k + 1] - it_[:, :7, :, k]
    v = float(np.median(d))
    tot += v
    print(f"  {labels[k]:40s} {v:8.0f}")
nxt = it_[:, :7, 1, 0] - it_[:, :7, 0, 9]
print(f"  {'item end -> next item start':40s} {float(np.median(nxt)):8.0f}")
print(f"  {'sum':40s} {tot:8.0f}")

# inside the item end: stamp 8 -> staging written (dK) -> stores issued (dK) -> staging (dV) -> stores (dV) -> K DMA
if hasattr(lib, "vit_diag_attn_xstamps"):
    xb = (ctypes.c_ulonglong * (16 * 8 * 2 * 8))()
    assert lib.vit_diag_attn_xstamps(xb, 16 * 8 * 2 * 8) == 0
    xs = np.frombuffer(xb, dtype=np.uint64).astype(np.int64).reshape(16, 8, 2, 8)
    seq = [it_[:, :7, :, 8], xs[:, :7, :, 1], xs[:, :7, :, 2], xs[:, :7, :, 3], xs[:, :7, :, 4], xs[:, :7, :, 0],
           it_[:, :7, :, 9]]
    names = ["dK staging writes", "dK row stores", "dV staging writes", "dV row stores", "(to K DMA)", "K DMA issue"]
    print("item end detail:")
    for k in range(6):
        print(f"  {names[k]:24s} {float(np.median(seq[k + 1] - seq[k])):8.0f}")
