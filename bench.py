"""Training-throughput benchmark: ViT-Base/16, 224x224, bf16, batch 256 per GPU (BASELINE.json configs[1]/[2]).

One step = the reference hot loop (train.py:89-96) on a synthetic batch already resident in HBM: fused forward,
softmax cross-entropy, zero_grad(set_to_none), backward (+ RCCL gradient all-reduce overlapped with it when N > 1),
FusedAdamW step.  Weak scaling: every rank processes its own batch of 256.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

Rank 0 prints ONE JSON line.  `roofline` is measured live: HIP events on the compute stream bracket every launch of
the dominant kernel family's representative GEMM (the fused QKV projection forward, M=B*T, N=3D, K=D: one launch of
gemm_bf16_v4<kcontig, kcontig, bf16, EPI_PLAIN>) inside the timed steps.
`cpu_baseline` times the oracle port (oracle/vit_oracle.py: the reference's algorithm restated in torch on CPU) on
the host cores, rank 0 at N=1 only, on a bounded sample (ViT-B/16 224^2 fp32, batch 8, 1 warmup + 3 steps).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16 = 2.5e15      # dense bf16 MFMA, MI355X (MI355X_MICROARCH.md chip table; no sparsity)
PEAK_F32 = 157.3e12     # fp32 MFMA


def gflop_per_image(D, L, T, N, P, C, nc):
    """Algorithmic fwd+bwd GFLOP per image: dense contractions only, patch-embed wgrad only."""
    pe = 2.0 * N * (C * P * P) * D
    block = 24.0 * T * D * D + 4.0 * T * T * D
    head = 2.0 * D * 4 * D + 2.0 * 4 * D * nc
    return (2 * pe + 3 * (L * block + head)) / 1e9


def pmc_traffic():
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 PMC passes (profiles/, FETCH_SIZE with
    the gfx950 x2 correction + WRITE_SIZE; tools/r2d.sh), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "r2_qkv_fwd_pmc.json")) as f:
            return int(json.load(f)["hbm_bytes_per_launch"])
    except (OSError, KeyError, ValueError):
        return None


def gemm_peak(dev, n=8192, reps=5):
    """Measured dense bf16 MFMA GEMM rate on this device: this library's GEMM and hipBLASLt
    (torch.matmul) on one n^3 GEMM of uniform [-1, 1) operands, outside the timed steps."""
    from VisionTransformer import _ops
    g = torch.Generator(device=dev).manual_seed(7)
    a = (torch.rand(n, n, device=dev, generator=g) * 2 - 1).bfloat16()
    b = (torch.rand(n, n, device=dev, generator=g) * 2 - 1).bfloat16()
    c = torch.empty(n, n, dtype=torch.bfloat16, device=dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / reps

    flop = 2.0 * n ** 3
    t_ours = timed(lambda: _ops.gemm(a, b, c, n, n, n, n, n, n))
    t_lib = timed(lambda: torch.matmul(a, b.t(), out=c))
    return {"shape": f"{n}x{n}x{n} bf16, uniform [-1,1)", "vit_gemm_tflops": round(flop / t_ours / 1e12, 1),
            "hipblaslt_tflops": round(flop / t_lib / 1e12, 1)}


def cpu_baseline(model_name, img, nc, batch=8, warmup=1, steps=3):
    from oracle import vit_oracle as O
    threads = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    ocfg = O.make_config(model_name, img=img, batch=batch, num_classes=nc)
    st = O.init_state(ocfg, seed=0)
    opt = O.AdamWState(st, lr=1e-4)
    x, y = O.synthetic_batch(ocfg)
    t0 = None
    for i in range(warmup + steps):
        if i == warmup:
            t0 = time.perf_counter()
        _, loss, grads = O.loss_and_grads(st, x, y, ocfg, train=True, seed=i)
        opt.step(st, grads)
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle/vit_oracle.py train step (fwd+CE+bwd+AdamW, dropout on), ViT-{model_name}/16 {img}^2 "
                      f"fp32, batch {batch}, {warmup} warmup + {steps} timed steps, {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="base", choices=["tiny", "small", "base", "large"])
    ap.add_argument("--img", type=int, default=224)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gemm-peak", action="store_true", help="skip the measured 8192^3 GEMM peak (profiling runs)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from VisionTransformer import config, vit
    from VisionTransformer.optim import FusedAdamW, cross_entropy

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    cfg = config.ViTConfig.preset(args.model, img_size=args.img, batch_size=args.batch, num_classes=args.classes,
                                  precision=dtype, device="cpu")
    torch.manual_seed(0)                       # identical init on every rank (reference init order, CPU RNG)
    model = vit.VisionTransformer(cfg).to(dev).train()
    if world > 1:
        model.enable_data_parallel()
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    gen = torch.Generator().manual_seed(1234 + rank)
    x = torch.randn(args.batch, 3, args.img, args.img, generator=gen).to(dev)
    y = torch.randint(0, args.classes, (args.batch,), generator=torch.Generator().manual_seed(1235 + rank)).to(dev)

    eng = model.hip_engine
    D, L, T, N = cfg.embedding_size, cfg.num_blocks, cfg.num_patches + 1, cfg.num_patches
    M = args.batch * T
    qkv_flop = 2.0 * M * 3 * D * D
    events = []

    def hook(name, phase):
        if name == "qkv_fwd":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            events.append(ev)

    def step():
        logits = model(x)
        loss = cross_entropy(logits, y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.profile_hook = hook
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    eng.profile_hook = None
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    final_loss = loss.item()
    kdur = [events[i].elapsed_time(events[i + 1]) / 1e3 for i in range(0, len(events) - 1, 2)]
    kavg = sum(kdur) / max(len(kdur), 1)

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        imgs = world * args.batch * args.steps / elapsed
        gf = gflop_per_image(D, L, T, N, cfg.patch_size, 3, args.classes)
        peak = PEAK_BF16 if dtype == torch.bfloat16 else PEAK_F32
        out = {
            "metric": "images/sec fwd+bwd ViT-Base/16 224^2 bf16 (train step incl. AdamW); % MFMA roofline",
            "value": round(imgs, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (N(0,1) images, uniform labels; random-init weights of the reference architecture)",
            "config": {"workload": f"ViT-{args.model.capitalize()}/16 {args.img}x{args.img} train step "
                                   f"(fwd+CE+bwd+AdamW), batch {args.batch}/GPU",
                       "model": f"vit_{args.model}_patch16_{args.img}", "global_batch": args.batch * world,
                       "seq_len": T, "parallelism": f"dp{world}"},
            "step_mfma_frac": round(imgs * gf * 1e9 / (world * peak), 4),
            "gflop_per_image": round(gf, 3),
            "final_loss": round(final_loss, 4),
            "roofline": {"bound": "mfma", "kernel": "gemm_bf16_v4<true,true,bf16,0> (fused QKV projection forward)",
                         "achieved": round(qkv_flop / kavg / 1e12, 2) if kavg > 0 else None,
                         "peak": peak / 1e12, "unit": "TFLOP/s",
                         "frac": round(qkv_flop / kavg / peak, 4) if kavg > 0 else None,
                         "flop_per_launch": qkv_flop, "avg_launch_us": round(kavg * 1e6, 2),
                         "launches_timed": len(kdur), "traffic": pmc_traffic(),
                         "traffic_source": "profiles/r2_qkv_fwd_pmc.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)"},
            "measured_gemm_peak": None if args.no_gemm_peak else gemm_peak(dev),
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.model, args.img, args.classes)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
