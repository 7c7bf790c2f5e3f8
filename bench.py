"""Training-throughput benchmark: ViT-Base/16, 224x224, bf16, batch 256 per GPU (BASELINE.json configs[1]/[2]).

One step = the reference hot loop (train.py:89-96) on a synthetic batch already resident in HBM: fused forward,
softmax cross-entropy, zero_grad(set_to_none), backward (+ RCCL gradient all-reduce overlapped with it when N > 1),
FusedAdamW step.  Weak scaling: every rank processes its own batch of 256.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

With `--gpus N > 1` and no torchrun environment, bench.py starts the N ranks itself (spawned children; the parent
makes no GPU call).  `--dry-run` replaces the HIP model by a CPU stand-in on gloo, to test the launch plumbing without
a GPU.  Rank 0 prints ONE JSON line.

Live roofline: HIP events on the compute stream bracket every hot launch of the last timed step, grouped into families
(forward / dgrad / wgrad GEMMs, attention fwd/bwd, LayerNorm fwd/bwd), each launch carrying its algorithmic FLOPs and
HBM bytes.  `roofline` reports the family that takes the most time; `roofline_families`
reports all of them.  `traffic` is the measured HBM bytes per launch of that family (rocprofv3 PMC passes under
profiles/ for this exact workload), or null when no such profile exists.
`cpu_baseline` times the repo's own host training step (train.py `time_steps`, VisionTransformer/_cpu.py) on all the
cores this process may use: BASELINE config 1 exactly (ViT-Tiny/16 64^2 B8 fp32, 5 warmup + 30 steps) and a bounded
ViT-Base/16 224^2 fp32 sample whose images/s is `value`.
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16 = 2.5e15      # dense bf16 MFMA, MI355X (MI355X_MICROARCH.md chip table; no sparsity)
PEAK_F32 = 157.3e12     # fp32 MFMA
PEAK_HBM = 8.0e12       # HBM3E bytes/s


def metric_name(args):
    """The headline metric string for this workload (BASELINE.json metric for ViT-Base/16 224^2 bf16)."""
    return (f"images/sec fwd+bwd ViT-{args.model.capitalize()}/16 {args.img}^2 {args.dtype} (train step incl. AdamW); "
            f"% MFMA roofline")


def gflop_per_image(D, L, T, N, P, C, nc):
    """Algorithmic fwd+bwd GFLOP per image: dense contractions only, patch-embed wgrad only."""
    pe = 2.0 * N * (C * P * P) * D
    block = 24.0 * T * D * D + 4.0 * T * T * D
    head = 2.0 * D * 4 * D + 2.0 * 4 * D * nc
    return (2 * pe + 3 * (L * block + head)) / 1e9


def gflop_executed_per_image(D, L, T, N, P, C, nc, pruned, row0=True):
    """GFLOP per image the kernels actually execute: the reference count minus what the pruned last block skips
    (its outputs and gradients are identical to the unpruned engine's, tested): proj / fc1 / fc2 (fwd,
    dgrad, wgrad: 54 D^2 per token) on the T-1 rows other than token 0, and its attention on queries other than 0
    (12 T^2 D fwd + bwd -> 14 T D for query 0 alone) with the Q third of its QKV GEMMs (fwd, dgrad, wgrad: 6 D^2 per
    token) on rows other than token 0 (round 5)."""
    full = gflop_per_image(D, L, T, N, P, C, nc)
    if not pruned:
        return full
    att = 12.0 * T * T * D - 14.0 * T * D + 6.0 * D * D * (T - 1) if row0 else 0.0
    return full - (54.0 * D * D * (T - 1) + att) / 1e9


def workload_key(args):
    return f"{args.model}_{args.img}_b{args.batch}_{args.dtype}"


def pmc_traffic(key, family):
    """Measured HBM bytes per step of `family` for this workload (profiles/pmc_<key>.json, written by
    tools/pmc_families.py from rocprofv3 PMC passes: FETCH_SIZE (x2 gfx950 correction) + WRITE_SIZE), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", f"pmc_{key}.json")) as f:
            fam = json.load(f)["families"][family]
        return int(fam["hbm_bytes_per_step"]), fam
    except (OSError, KeyError, ValueError, TypeError):
        return None, None


def pmc_schedule(key):
    """The schedule the PMC passes of profiles/pmc_<key>.json ran (tools/gpu_profile.sh), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", f"pmc_{key}.json")) as f:
            return json.load(f).get("schedule", "default (two forward chains + weight-gradient stream)")
    except (OSError, ValueError):
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


def log(msg):
    """Progress on stderr (a long silent run looks hung to the GPU box's watchdog)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def host_topology():
    """CPUs this process may use (its affinity mask), the machine's OMP_NUM_THREADS share when one is set (the GPU
    box exports 16 per GPU), plus sockets / physical cores of the host (/proc/cpuinfo)."""
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    sockets, cores = set(), set()
    try:
        phys = core = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":")[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":")[1].strip()
                elif not line.strip() and phys is not None:
                    sockets.add(phys)
                    cores.add((phys, core))
                    phys = core = None
    except OSError:
        pass
    quota = None                                   # cgroup v2 CPU bandwidth limit (e.g. "1600000 100000" = 16 CPUs)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    usable = min(affinity, quota) if quota else affinity
    return {"affinity_cpus": affinity, "cgroup_cpu_quota": quota, "usable_cpus": usable,
            "omp_num_threads": share or None, "host_logical_cpus": os.cpu_count(),
            "sockets": len(sockets) or None, "physical_cores": len(cores) or None}


def _cpu_leg(img, nc, threads, budget_s):
    """C1 exactly (ViT-Tiny/16 64^2 B8 fp32, 5 warmup + 30 timed steps), then ViT-Base/16 img^2 fp32 B32: 1 warmup
    step, then as many timed steps (1-3) as fit in ~budget_s, on `threads` threads."""
    import train as T
    from VisionTransformer import config
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        c1 = config.ViTConfig(3, 10, 16, 192, 16, 3, 12, "cpu", 8)
        log(f"cpu baseline: C1 on {threads} threads")
        s1, _ = T.time_steps(c1, steps=30, warmup=5, dev="cpu")
        log(f"cpu baseline: C1 {s1 * 1e3:.1f} ms/step; ViT-B B32 warmup step")
        cb = config.ViTConfig.preset("base", img_size=img, batch_size=32, num_classes=nc, precision=torch.float32,
                                     device="cpu")
        t0 = time.perf_counter()
        T.time_steps(cb, steps=0, warmup=1, dev="cpu")
        one = time.perf_counter() - t0
        steps = int(max(1, min(3, budget_s // max(one, 1e-3))))
        log(f"cpu baseline: ViT-B step {one:.1f} s; timing {steps} step(s)")
        sb, _ = T.time_steps(cb, steps=steps, warmup=1, dev="cpu")
    finally:
        torch.set_num_threads(prev)
    return {"images_per_s": round(32 / sb, 3), "steps": steps, "threads": threads,
            "c1": {"workload": "BASELINE config 1: ViT-Tiny/16 64^2 B8 fp32, 5 warmup + 30 timed steps",
                   "ms_per_step": round(s1 * 1e3, 3), "images_per_s": round(8 / s1, 3)}}


def cpu_baseline(img, nc, budget_s=20.0):
    """The repo's own CPU training step (train.py time_steps -> VisionTransformer/_cpu.py, torch.optim.AdamW) on every
    CPU this process can use: its affinity mask, capped by the cgroup CPU quota when one is set (the GPU box shows
    256 affinity CPUs but grants a 16-CPU quota; 256 threads on 16 CPUs time-slice each other to a standstill).  Also
    on the box's OMP_NUM_THREADS share when that is smaller (`share`)."""
    topo = host_topology()
    n = topo["usable_cpus"]
    full = _cpu_leg(img, nc, n, budget_s)
    why = "every CPU of the affinity mask" if n == topo["affinity_cpus"] else \
        f"the cgroup CPU quota ({n} of {topo['affinity_cpus']} affinity CPUs)"
    out = {"value": full["images_per_s"], "unit": "images/s", "cores": full["threads"], "kind": "port",
           "sample": f"repo train.py host step (VisionTransformer/_cpu.py fwd+CE+bwd + torch AdamW, dropout on), "
                     f"ViT-Base/16 {img}^2 fp32 B32, 1 warmup + {full['steps']} timed steps, "
                     f"{full['threads']} threads ({why})",
           "topology": topo, "c1": full["c1"]}
    share = topo["omp_num_threads"]
    if share and share < n:
        sh = _cpu_leg(img, nc, share, budget_s)
        out["share"] = {"threads": share, "images_per_s": sh["images_per_s"], "c1": sh["c1"],
                        "note": "the GPU box's OMP_NUM_THREADS share per GPU"}
    return out


class FamilyTimer:
    """HIP events around every hot launch (engine.profile_hook), grouped by kernel family."""

    def __init__(self):
        self.open = {}
        self.done = []          # (family, start, end, flop, bytes)

    def __call__(self, fam, phase, flop=0.0, nbytes=0.0):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        if phase == 0:
            self.open[fam] = (ev, flop, nbytes)
        else:
            s, f, b = self.open.pop(fam)
            self.done.append((fam, s, ev, f, b))

    def summary(self, steps):
        fams = {}
        for fam, s, e, f, b in self.done:
            d = fams.setdefault(fam, {"launches": 0, "time_s": 0.0, "flop": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["time_s"] += s.elapsed_time(e) / 1e3
            d["flop"] += f
            d["bytes"] += b
        out = {}
        for fam, d in fams.items():
            t = max(d["time_s"], 1e-12)
            out[fam] = {"launches_per_step": d["launches"] // steps, "ms_per_step": round(d["time_s"] / steps * 1e3, 3),
                        "avg_launch_us": round(t / d["launches"] * 1e6, 2),
                        "tflops": round(d["flop"] / t / 1e12, 2), "hbm_gbs_algorithmic": round(d["bytes"] / t / 1e9, 1),
                        "flop_per_step": d["flop"] / steps, "bytes_per_step": d["bytes"] / steps}
        return out


def run(args, rank, world, local):
    if args.dry_run:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    if args.dry_run:          # launch-plumbing stand-in: one small CPU GEMM + a gradient-sized all-reduce per step
        w = torch.randn(256, 256)
        g = torch.zeros(1 << 16)
        comm_ms = [None]

        def step():
            y = (w @ w).sum()
            if world > 1:
                t = time.perf_counter()
                dist.all_reduce(g)
                comm_ms[0] = (time.perf_counter() - t) * 1e3      # the stand-in's all-reduce is fully exposed
            return y
        D = L = T = N = 0
        cfg = None
    else:
        from VisionTransformer import _lib, config, vit
        from VisionTransformer.optim import FusedAdamW, cross_entropy
        for kv in args.opt:
            name, val = kv.split("=")
            _lib.set_option(name, int(val))
        cfg = config.ViTConfig.preset(args.model, img_size=args.img, batch_size=args.batch, num_classes=args.classes,
                                      precision=dtype, device="cpu")
        torch.manual_seed(0)                       # identical init on every rank (reference init order, CPU RNG)
        model = vit.VisionTransformer(cfg).to(dev).train()
        for kv in args.engine:
            name, val = kv.split("=")
            if not hasattr(model.hip_engine, name):
                raise SystemExit(f"--engine: no Engine attribute {name!r}")
            setattr(model.hip_engine, name, bool(int(val)) if isinstance(getattr(model.hip_engine, name), bool)
                    else int(val))
        if world > 1:
            model.enable_data_parallel(grad_dtype=torch.bfloat16 if args.grad_comm == "bf16" else torch.float32,
                                       launch_mode=args.launch_mode)
        opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
        gen = torch.Generator().manual_seed(1234 + rank)
        x = torch.randn(args.batch, 3, args.img, args.img, generator=gen).to(dev)
        y = torch.randint(0, args.classes, (args.batch,), generator=torch.Generator().manual_seed(1235 + rank)).to(dev)
        D, L, T, N = cfg.embedding_size, cfg.num_blocks, cfg.num_patches + 1, cfg.num_patches

        def step():
            logits = model(x)
            loss = cross_entropy(logits, y)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            return loss

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    if args.roctx and not args.dry_run:
        model.hip_engine.trace_ranges = True
    log(f"rank {rank}/{world}: warmup {args.warmup} steps")
    for _ in range(args.warmup):
        loss = step()
    sync()
    log(f"rank {rank}/{world}: timing {args.steps} steps")
    if world > 1:
        dist.barrier()
    sync()
    # The live roofline brackets every hot launch of the LAST timed step with HIP events (each event record is a
    # stream barrier: on every step they cost ~1.4 ms of the ~36 ms step, measured; on one step of K they cost ~1.4/K)
    timer = FamilyTimer() if not args.dry_run and not args.no_roofline else None
    roof_steps = 1 if timer is not None else 0
    t0 = time.perf_counter()
    conc = None if args.dry_run else model.hip_engine.concurrent_wgrad
    for i in range(args.steps):
        if timer is not None and i == args.steps - roof_steps:
            model.hip_engine.profile_hook = timer
            # the event-bracketed step runs the in-order schedule: with the weight gradients on their side stream the
            # backward families' events would time kernels sharing the GPU (the forward families are unaffected)
            model.hip_engine.concurrent_wgrad = False
        if world > 1 and not args.dry_run and i == args.steps - 1:
            model.hip_engine.time_comm = True         # events around the bucket waits of the last step
        loss = step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t1 = time.perf_counter()
    if timer is not None:
        model.hip_engine.profile_hook = None
        model.hip_engine.concurrent_wgrad = conc
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    comm = None
    if world > 1:
        # exposed all-reduce time of the last timed step (compute stream idle after its last backward kernel until
        # the last bucket is averaged), max over ranks
        c = comm_ms[0] if args.dry_run else model.hip_engine.comm_exposed_ms()
        if not args.dry_run:
            model.hip_engine.time_comm = False
        ct = torch.tensor([c if c is not None else -1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(ct, op=dist.ReduceOp.MAX)
        comm = float(ct.item()) if ct.item() >= 0 else None
    final_loss = float(loss.item())
    log(f"rank {rank}/{world}: {elapsed / args.steps * 1e3:.2f} ms/step")

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        imgs = world * args.batch * args.steps / elapsed
        out = {
            "metric": metric_name(args),
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
        }
        if args.opt:
            out["options"] = dict(kv.split("=") for kv in args.opt)
        if args.engine:
            out["engine"] = dict(kv.split("=") for kv in args.engine)
        if world > 1:
            out["comm_exposed_ms"] = round(comm, 3) if comm is not None else None
            out["grad_comm_dtype"] = args.grad_comm
            out["launch_mode"] = args.launch_mode
        if args.dry_run:
            out["dry_run"] = True
            out["data"] = "dry run: CPU stand-in step on gloo, no HIP model (launch plumbing only)"
        else:
            gf = gflop_per_image(D, L, T, N, cfg.patch_size, 3, args.classes)
            peak = PEAK_BF16 if dtype == torch.bfloat16 else PEAK_F32
            out["step_mfma_frac"] = round(imgs * gf * 1e9 / (world * peak), 4)
            out["gflop_per_image"] = round(gf, 3)
            eng = model.hip_engine
            gfx = gflop_executed_per_image(D, L, T, N, cfg.patch_size, 3, args.classes, eng.prune_last,
                                           eng.row0_attention)
            out["step_mfma_frac_executed"] = round(imgs * gfx * 1e9 / (world * peak), 4)
            out["gflop_executed_per_image"] = round(gfx, 3)
            out["final_loss"] = round(final_loss, 4)
            if timer is not None:
                fams = timer.summary(roof_steps)
                dom = max(fams, key=lambda f: fams[f]["ms_per_step"])
                d = fams[dom]
                key = workload_key(args)
                traffic, pmc = pmc_traffic(key, dom)
                if dom.startswith("gemm") or dom.startswith("attn"):
                    ach, pk, unit, bound = d["tflops"], peak / 1e12, "TFLOP/s", "mfma"
                else:
                    ach, pk, unit, bound = d["hbm_gbs_algorithmic"], PEAK_HBM / 1e9, "GB/s", "hbm"
                out["roofline"] = {
                    "bound": bound, "family": dom, "achieved": ach, "peak": pk, "unit": unit,
                    "frac": round(ach / pk, 4),
                    "frac_basis": "FLOPs the family's launches execute (the pruned last block charged for its B "
                                  "token-0 rows only)" if bound == "mfma" else "algorithmic bytes",
                    # whole step, executed FLOPs (step_mfma_frac credits the reference's FLOPs, pruned rows included)
                    "step_frac_executed": out["step_mfma_frac_executed"],
                    # per launch, like `achieved`: the PMC family's HBM bytes per step / this family's launches
                    "traffic": int(traffic / d["launches_per_step"]) if traffic is not None else None,
                    "traffic_unit": "HBM bytes per launch (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE)",
                    "traffic_per_step": traffic,
                    "algorithmic_bytes_per_launch": int(d["bytes_per_step"] / d["launches_per_step"]),
                    "algorithmic_bytes_per_step": int(d["bytes_per_step"]),
                    "pmc_mfma_busy_frac": pmc.get("mfma_busy_frac") if pmc else None,
                    "pmc_schedule": pmc_schedule(key),
                    "traffic_source": f"profiles/pmc_{key}.json" if traffic is not None else None,
                    "ms_per_step": d["ms_per_step"], "launches_per_step": d["launches_per_step"],
                    "events_over": "every hot launch of the last of the timed steps (HIP events on the compute stream)",
                    "avg_launch_us": d["avg_launch_us"],
                    "kernels": family_kernels(dom)}
                for f, v in fams.items():
                    pk_f = peak if (f.startswith("gemm") or f.startswith("attn")) else None
                    v["mfma_frac"] = round(v["tflops"] * 1e12 / peak, 4) if pk_f else None
                    v["hbm_frac_algorithmic"] = round(v["hbm_gbs_algorithmic"] * 1e9 / PEAK_HBM, 4)
                    del v["flop_per_step"], v["bytes_per_step"]
                out["roofline_families"] = fams
            if not args.no_gemm_peak:
                log("measured GEMM peak")
                out["measured_gemm_peak"] = gemm_peak(dev)
        if world == 1 and not args.no_cpu_baseline and not args.dry_run:
            out["cpu_baseline"] = cpu_baseline(args.img, args.classes)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def family_kernels(fam):
    """The kernels a roofline family's HIP events time (what `roofline.kernels` names): every launch between the
    engine's family marks, the split-K pieces included."""
    main = "gemm_bf16_v4"
    slab = "gemm_bf16_v4<*,*,float,EPI_SLAB> + splitk_reduce"
    return {"gemm_wgrad": f"gemm_bf16_v4<false,false,float,EPI_SLAB> + splitk_reduce<float>",
            "gemm_fwd": f"{main}<true,true,bf16,*> (patch embedding: gemm_bf16_v4 EPI_PATCH) + the N=768 / K>=2304 "
                        f"split-K tail and the pruned last block's split-K launches: {slab}",
            "gemm_dgrad": f"{main}<true,false,*> + the split-K tail and the pruned last block's split-K launches: "
                          f"{slab}",
            "attn_fwd": "attn_fwd_fused / attn_fwd_mfma", "attn_bwd": "attn_bwd_fused / attn_bwd_dq_mfma + "
                                                                      "attn_bwd_dkdv_mfma",
            "ln_fwd": "ln_fwd16_kernel / ln_fwd_kernel", "ln_bwd": "ln_bwd_kernel"}.get(fam, fam)


def _spawned(rank, args, world, port):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run(args, rank, world, rank)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="base", choices=["tiny", "small", "base", "large"])
    ap.add_argument("--img", type=int, default=224)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--grad-comm", default="fp32", choices=["fp32", "bf16"],
                    help="dtype of the gradient all-reduce buckets for N > 1 (bf16: half the xGMI bytes)")
    ap.add_argument("--launch-mode", default="auto", choices=["auto", "shared", "persistent"],
                    help="N > 1: backward kernels beside RCCL as persistent one-per-CU grids (persistent; auto) or "
                         "one workgroup per item (shared) (DESIGN.md 5.4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gemm-peak", action="store_true", help="skip the measured 8192^3 GEMM peak (profiling runs)")
    ap.add_argument("--no-roofline", action="store_true", help="no per-launch HIP events (profiling runs)")
    ap.add_argument("--roctx", action="store_true",
                    help="roctx ranges per kernel family (rocprofv3 --marker-trace timelines; costs host time)")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo stand-in step: tests rank launch without a GPU")
    ap.add_argument("--engine", action="append", default=[], metavar="ATTR=INT",
                    help="set an Engine attribute for A/B runs (e.g. row0_attention=0, prune_last=0)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="library launch option (vit_set_option; A/B runs of kernel variants, default: shipped)")
    args = ap.parse_args(argv)

    if "WORLD_SIZE" in os.environ:           # launched by torchrun: one rank per process
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; using WORLD_SIZE", file=sys.stderr)
        run(args, int(os.environ.get("RANK", "0")), world, int(os.environ.get("LOCAL_RANK", "0")))
    elif args.gpus > 1:                      # start the ranks here; this parent makes no GPU call
        import torch.multiprocessing as mp
        mp.start_processes(_spawned, args=(args, args.gpus, _free_port()), nprocs=args.gpus, start_method="spawn")
    else:
        run(args, 0, 1, 0)


if __name__ == "__main__":
    main()
