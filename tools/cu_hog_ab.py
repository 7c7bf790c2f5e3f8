"""Persistent grids vs the shared-CU launch mode when other kernels hold CUs (one GPU, no collective).

At N > 1 RCCL's all-reduce kernels run beside the backward: each bucket's all-reduce (launched when the block's last
weight gradient is enqueued, `_engine._bucket_ready`) holds some CUs for a while.  The backward's bf16 GEMMs and the
fused attention backward normally run a persistent grid (one workgroup per CU, items assigned statically), where a
workgroup whose CU is held waits, and its items with it; `enable_data_parallel()` on nccl therefore switches them to
one workgroup per item (VIT_FLAG_SHARED_CUS).  This tool measures both modes on one GPU with a stand-in for the
collective: at every bucket it launches `tools/micro/cu_hog.hip` (NWG workgroups that each hold a CU for US
microseconds) on a side stream that waits for the compute stream, and the compute stream waits for it before the
optimizer, as for the real all-reduce.

    python tools/cu_hog_ab.py [--nwg 32 64] [--us 400] [--rounds 2]

Prints one line per (mode, hog) with ms/step and the time the compute stream waited for the last hog after its last
backward kernel (the stand-in for exposed all-reduce time); `--nwg 0` is the no-hog baseline."""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nwg", type=int, nargs="+", default=[0, 32, 64])
    ap.add_argument("--threads", type=int, default=256)
    ap.add_argument("--us", type=float, default=400.0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()

    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "micro", "libcu_hog.so"))
    lib.cu_hog_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
    lib.cu_hog_launch.restype = ctypes.c_int

    from VisionTransformer import config, vit
    from VisionTransformer.optim import FusedAdamW, cross_entropy
    dev = torch.device("cuda", 0)
    cfg = config.ViTConfig.preset("base", img_size=224, batch_size=args.batch, num_classes=1000,
                                  precision=torch.bfloat16, device="cpu")
    torch.manual_seed(0)
    model = vit.VisionTransformer(cfg).to(dev).train()
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    x = torch.randn(args.batch, 3, 224, 224, generator=torch.Generator().manual_seed(1)).to(dev)
    y = torch.randint(0, 1000, (args.batch,), generator=torch.Generator().manual_seed(2)).to(dev)
    eng = model.hip_engine
    side = torch.cuda.Stream(dev)
    sink = torch.zeros(1024, device=dev)
    state = {"nwg": 0, "pending": False, "events": []}

    def bucket_ready(rng, side_stream=None):
        if state["nwg"] == 0:
            return
        side.wait_stream(torch.cuda.current_stream(dev))
        rc = lib.cu_hog_launch(state["nwg"], args.threads, args.us, ctypes.c_void_p(sink.data_ptr()),
                               ctypes.c_void_p(side.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"cu_hog_launch rc={rc}")
        state["pending"] = True

    def finish_buckets():
        if state["pending"]:
            cur = torch.cuda.current_stream(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)                  # every backward kernel is enqueued before this point
            cur.wait_stream(side)
            e1.record(cur)
            state["events"].append((e0, e1))
            state["pending"] = False

    eng._bucket_ready = bucket_ready
    eng._finish_buckets = finish_buckets

    def step():
        logits = model(x)
        loss = cross_entropy(logits, y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    def timed(shared, nwg):
        eng.shared_cus = shared
        state["nwg"] = nwg
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t) / args.steps * 1e3
        ev = state["events"][-args.steps:]
        exposed = sum(a.elapsed_time(b) for a, b in ev) / len(ev) if ev else 0.0
        state["events"] = []
        return ms, exposed

    print(f"ViT-B/16 224 B{args.batch} bf16 train step; hog = NWG workgroups x {args.threads} threads holding a CU for "
          f"{args.us:.0f} us at each of the {eng.L + 2} gradient buckets", flush=True)
    for r in range(args.rounds):
        for nwg in args.nwg:
            for shared in (False, True):
                ms, exposed = timed(shared, nwg)
                mode = "shared-CU (one WG per item)" if shared else "persistent (one WG per CU)"
                print(f"round {r} hog {nwg:4d} WGs  {mode:30s} {ms:8.3f} ms/step   hog still running after the "
                      f"last backward kernel: {exposed:6.3f} ms", flush=True)


if __name__ == "__main__":
    main()
