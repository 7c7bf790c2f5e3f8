"""Per-tile time breakdown of the v4 GEMM from a diagnostic build with in-kernel s_memtime stamps.

    tools/build_variant.sh stamps vision-transformer_amd/csrc/vit_gemm.hip -DVIT_GEMM_STAMPS
    python tools/gemm_stamps.py tools/variants/libvit_hip_stamps.so [--shapes fwd_fc1m,...]

Each workgroup accumulates the shader-clock cycles of each interval over the items it processes (vit_gemm.hip,
V4_ACC): k-loop, next-tile stage issue, epilogue, restage + wait, loop-top barrier, first prologue, and the tail.
Prints, over workgroups, the median per item of each interval.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
import torch  # noqa: E402
import gemm_ab  # noqa: E402

NAMES = ["k-loop", "next-issue", "epilogue", "restage+wait", "top-barrier", "first-prologue", "items", "tail"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--shapes", default="fwd_qkv,fwd_fc1m,fwd_fc2,dgrad_fc2m")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    lib = gemm_ab.load(args.lib)
    lib.vit_gemm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ws = torch.empty(96 << 20, dtype=torch.float32, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    buf = np.zeros(16384 * 8, dtype=np.uint64)
    for sname in args.shapes.split(","):
        m, n, k, akc, bkc, epi = gemm_ab.SHAPES[sname]
        a = (torch.rand((m, k) if akc else (k, m), device="cuda", generator=g) * 2 - 1).bfloat16()
        b = (torch.rand((n, k) if bkc else (k, n), device="cuda", generator=g) * 2 - 1).bfloat16()
        aux = (torch.rand(m, n, device="cuda", generator=g) - 0.3).bfloat16()
        res = torch.randn(m, n, device="cuda", generator=g).bfloat16()
        bias = torch.randn(n, device="cuda", generator=g)
        mask = torch.randint(0, 256, (4 * ((m + 3) // 4) * ((n + 3) // 4),), device="cuda", generator=g,
                             dtype=torch.uint8)
        c = torch.empty(m, n, dtype=torch.float32 if epi == "wgrad" else torch.bfloat16, device="cuda")
        split = lib.vit_gemm_split_k_hint(m, n, k, gemm_ab._lib.BF16) if epi == "wgrad" else 1
        d = gemm_ab.desc(a, b, c, m, n, k, akc, bkc, epi, split, ws, aux, bias, res, mask)
        buf[:] = 0
        lib.vit_gemm_debug_stamps_reset()
        walls = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert lib.vit_gemm(ctypes.byref(d), stream) == 0
            e1.record()
            torch.cuda.synchronize()
            walls.append(e0.elapsed_time(e1) * 1e-3)
        assert lib.vit_gemm_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
        st = buf.reshape(-1, 8).astype(np.int64)
        st = st[st[:, 6] > 0]                              # workgroups that ran (persistent grids: one per CU)
        items = st[:, 6].astype(np.float64)
        wall = sorted(walls)[len(walls) // 2]
        tot = st[:, [0, 1, 2, 3, 4, 5, 7]].sum(1)
        print(f"{sname:10s} wgs={len(st):5d} items/wg med={np.median(items):.1f} wall={wall * 1e6:7.1f}us "
              f"cycles/wg med={np.median(tot):8.0f} -> {np.median(tot) / wall / 1e9:.2f} GHz", flush=True)
        for k, nm in enumerate(NAMES):
            if nm == "items":
                continue
            per = st[:, k] / items
            print(f"    {nm:14s} per item med {np.median(per):8.0f}  p10 {np.percentile(per, 10):8.0f}  p90 "
                  f"{np.percentile(per, 90):8.0f} cyc", flush=True)
        buf[:] = 0


if __name__ == "__main__":
    main()
