"""Training entry point — drop-in for the reference's src/train.py (run from this directory, like the reference).

Same public functions: `evaluate(model, test_loader, eval_func, avg=None)` (train.py:29-44),
`search_checkpoint(dir)` (:52-58), `train(configs, train_loader, test_loader, epochs, eval_iter, log_dir,
checkpoint_dir, lr=1e-4)` (:60-119), and the same checkpoint dict {epoch, model_state_dict, optimizer_state_dict,
loss, step} (:107-113), so checkpoints interchange with the reference (per-head state_dict keys, torch AdamW state
keys).  The hot loop (:89-102) runs on the MI355X path: fused HIP forward/backward, fused softmax cross-entropy,
FusedAdamW (one multi-tensor launch), and — under torchrun — gradient all-reduce over RCCL overlapped with the
backward.  The per-step `loss.item()` host sync of the reference is kept only when logging asks for it.
Without a GPU (or with `--device cpu`) the same loop runs the package's host path (VisionTransformer/_cpu.py, plain
torch ops on all host cores, torch.optim.AdamW) — the reference's own behaviour (train.py:26,80) and BASELINE config 1
(ViT-Tiny/16 64^2 B8 fp32, `python train.py --device cpu`).

Differences (documented in DESIGN.md): hyper-parameters come from flags instead of hard-coded constants (the
reference's TODO at :124-125); data defaults to a synthetic CIFAR-shaped stream because the container has no network
(CIFAR10(download=True) at :157-159 cannot run).  `--data cifar10-bin --data-root R` reads CIFAR-10's binary batches,
`--data folder --data-root R` a folder-per-class image tree (BrainTumorDataset.py), `--data synthetic-u8` random uint8
images; on the GPU those run the reference transform (convert RGB -> Resize((S, S)) -> ToTensor, train.py:151-155)
as one kernel per batch (VisionTransformer/data.py, bit-exact with Pillow), on the host with Pillow per image.
tensorboard is used when importable, else scalars go to a JSONL file.
"""
import argparse
import glob
import json
import os
import re
import time

import torch
import torch.distributed as dist

from VisionTransformer import config, vit
from VisionTransformer.optim import cross_entropy, make_optimizer

device = "cuda" if torch.cuda.is_available() else "cpu"


class _JsonlWriter:
    """Minimal stand-in for tensorboard's SummaryWriter (tensorboard is not installed in this image)."""

    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.f = open(os.path.join(log_dir, "scalars.jsonl"), "a")

    def add_scalar(self, tag, value, step):
        self.f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step), "t": time.time()}) + "\n")
        self.f.flush()


def _writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=log_dir, flush_secs=10)
    except Exception:
        return _JsonlWriter(log_dir)


class ShardSampler(torch.utils.data.Sampler):
    """Rank `rank` of `world` reads indices rank, rank + world, ... < n in order: the shards partition the set exactly
    (DistributedSampler instead pads every shard to equal length with duplicates), so a sharded evaluate() scores
    every test sample once."""

    def __init__(self, dataset, rank=None, world=None):
        r, w = _rank_world()
        self.n = len(dataset)
        self.rank = r if rank is None else rank
        self.world = w if world is None else world

    def __iter__(self):
        return iter(range(self.rank, self.n, self.world))

    def __len__(self):
        return len(range(self.rank, self.n, self.world))


def _sampler_of(loader):
    for obj in (loader, getattr(loader, "loader", None)):
        if obj is None:
            continue
        for s in (getattr(obj, "sampler", None), getattr(getattr(obj, "batch_sampler", None), "sampler", None)):
            if isinstance(s, (torch.utils.data.DistributedSampler, ShardSampler)):
                return s
    return None


@torch.no_grad()
def evaluate(model, test_loader, eval_func, avg=None):
    """Mean over batches of eval_func(labels, argmax(logits)) (train.py:29-44).

    A partial last batch is padded to the model's batch size (the CLS parameter is batch-shaped, vit.py:32,41) and
    only its real rows are scored; the reference would raise there.  With such a batch the score is eval_func over
    the whole set (every sample weighted once, the same value a data-parallel run returns) instead of the mean of
    per-batch scores, which is kept whenever every batch is full (the reference's only working case).

    Under data parallelism (an initialized process group of world size > 1) every rank scores its own shard of the test
    set, the (label, prediction) pairs of all ranks are gathered, and eval_func runs once over the whole set, so every
    rank returns the same score — for accuracy, the exact whole-set accuracy.  Each sample counts once: a ShardSampler
    shard has no duplicates, and the padding duplicates DistributedSampler appends (the trailing samples of a shard
    whose global position is >= len(dataset)) are dropped."""
    model.eval()
    score = 0.0
    n = 0
    labs, preds = [], []
    pad_to = getattr(getattr(model, "vit_config", None), "batch_size", None)
    for tensors, labels in test_loader:
        rows = tensors.shape[0]
        if pad_to is not None and rows < pad_to:
            fill = tensors[-1:].expand(pad_to - rows, *tensors.shape[1:])
            tensors = torch.cat([tensors, fill], 0)
        logits = model(tensors.to(device, non_blocking=True))[:rows]
        predictions = torch.argmax(logits, axis=-1).to("cpu")
        labels = labels.to("cpu")
        labs.append(labels)
        preds.append(predictions)
        if avg is None:
            score += eval_func(labels, predictions)
        else:
            score += eval_func(labels, predictions, average=avg, zero_division=0.0)
        n += 1
    model.train()
    rank, world = _rank_world()
    lab = torch.cat(labs) if labs else torch.zeros(0, dtype=torch.long)
    pred = torch.cat(preds) if preds else torch.zeros(0, dtype=torch.long)
    if world == 1:
        if pad_to is None or all(len(v) == pad_to for v in labs):
            return score / max(n, 1)             # the reference's mean of per-batch scores (full batches only)
        # a padded partial batch: score the whole set once, as the data-parallel case does, so the same model reports
        # the same score on one rank and on many (a mean of per-batch scores would weight the partial batch fully)
        if avg is None:
            return float(eval_func(lab, pred))
        return float(eval_func(lab, pred, average=avg, zero_division=0.0))
    s = _sampler_of(test_loader)
    if isinstance(s, torch.utils.data.DistributedSampler) and not s.drop_last:
        keep = len(range(rank, len(s.dataset), world))           # the shard's samples before the padding
        lab, pred = lab[:keep], pred[:keep]
    gathered = [None] * world
    dist.all_gather_object(gathered, (lab.tolist(), pred.tolist()))
    all_lab = torch.tensor([v for g in gathered for v in g[0]], dtype=torch.long)
    all_pred = torch.tensor([v for g in gathered for v in g[1]], dtype=torch.long)
    if avg is None:
        return float(eval_func(all_lab, all_pred))
    return float(eval_func(all_lab, all_pred, average=avg, zero_division=0.0))


def _set_epoch(loader, epoch):
    """DistributedSampler.set_epoch on the loader's sampler (also behind data.DeviceBatches), so each epoch draws a
    new shard order on every rank."""
    for obj in (loader, getattr(loader, "loader", None)):
        if obj is None:
            continue
        for s in (getattr(obj, "sampler", None), getattr(getattr(obj, "batch_sampler", None), "sampler", None)):
            if isinstance(s, torch.utils.data.DistributedSampler):
                s.set_epoch(epoch)
                return True
    return False


def search_checkpoint(dir):
    """Highest N of the N.pt files in dir, or None (train.py:52-58)."""
    epochs = glob.glob(os.path.join(dir, "*.pt"))
    if len(epochs) == 0:
        return None
    names = [os.path.basename(e) for e in epochs]
    nums = [int(m.group(1)) for m in (re.match(r"(\d+)(?=\.pt)", nm) for nm in names) if m]
    return max(nums) if nums else None


class SyntheticImages(torch.utils.data.Dataset):
    """Deterministic N(0,1) images with uniform labels (the bench/parity input distribution)."""

    def __init__(self, n, channels, img, classes, seed):
        self.n, self.shape, self.classes, self.seed = n, (channels, img, img), classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        return torch.randn(self.shape, generator=g), int(torch.randint(0, self.classes, (1,), generator=g))


def replica_seed(rank, base=0):
    """CPU RNG seed of data-parallel replica `rank` after the identically seeded init (host path): rank 0 keeps
    `base`, so a one-rank job draws what a plain run draws."""
    return base if rank == 0 else (base + 0x9E3779B1 * rank) % (2 ** 63 - 1)


def _rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def train(configs, train_loader, test_loader, epochs, eval_iter, log_dir, checkpoint_dir, lr=1e-4,
          log_every=1, max_steps=None, reference_loop=False):
    """The reference training loop (train.py:60-119) on the HIP path.  Returns the last epoch's summed loss.

    Defaults keep the GPU busy: no host sync inside the epoch — the epoch loss is summed on the device and the per-step
    "Loss/train_batch" scalars (every `log_every` steps, train.py:98) stay on the device until the epoch ends, when they
    are written in one transfer; validation runs every `eval_iter` epochs and a resumed run continues its step counter.
    `reference_loop=True` restores the reference's bookkeeping exactly: validation after every epoch (its eval_iter
    gate is commented out, train.py:114), `iteration` restarting at 0 on resume (train.py:67; the checkpoint's `step`
    is not read back) and the epoch loss as the host sum of each step's loss.item() (train.py:97-99: one host sync
    per step).  Under data parallelism a DistributedSampler gets `set_epoch(epoch)` every epoch and `evaluate`
    all-reduces its counts."""
    rank, world = _rank_world()
    saved_epoch = search_checkpoint(checkpoint_dir)
    torch.manual_seed(0)                              # identical init on every rank
    model = vit.VisionTransformer(configs)
    optimizer = make_optimizer(model.parameters(), lr=lr, weight_decay=1e-4, device=device)
    iteration = 0
    if saved_epoch is not None:
        print(f"Checkpoint Found. Loading model from epoch {saved_epoch}")
        ckpt = torch.load(os.path.join(checkpoint_dir, f"{saved_epoch}.pt"), map_location="cpu", weights_only=True)
        model.load_state_dict(ckpt["model_state_dict"])
        model = model.to(device)
        optimizer = make_optimizer(model.parameters(), lr=lr, weight_decay=1e-4, device=device)
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])
        iteration = 0 if reference_loop else int(ckpt.get("step", 0))
    else:
        saved_epoch = 0
        model = model.to(device)
    net = model
    if world > 1:
        if device == "cpu":      # host path: standard autograd, so torch's own DDP (gloo) applies
            net = torch.nn.parallel.DistributedDataParallel(model)
            # the host dropout (F.dropout, transformer.py:47,59) draws from the CPU RNG, seeded identically above
            # for identical init: give each replica its own stream, or all ranks mask their images alike
            torch.manual_seed(replica_seed(rank))
        else:
            model.enable_data_parallel()      # the engine folds the rank into its dropout seed
    writer = _writer(log_dir) if rank == 0 else None
    running_loss = 0.0
    for epoch in range(saved_epoch, epochs + 1):
        _set_epoch(train_loader, epoch)
        loss_sum = torch.zeros((), device=device)
        host_loss = 0.0
        logged = []                                   # (iteration, device loss) written at the epoch's end
        t0 = time.time()
        nb = 0
        for tensors, labels in train_loader:
            tensors = tensors.to(device, non_blocking=True)
            labels = labels.to(device, non_blocking=True)
            logits = net(tensors)
            loss = cross_entropy(logits, labels)
            optimizer.zero_grad(set_to_none=True)
            loss.backward()
            optimizer.step()
            if reference_loop:
                host_loss += loss.item()
                if writer is not None:
                    writer.add_scalar("Loss/train_batch", loss.item(), iteration)
            else:
                loss_sum += loss.detach()
                if writer is not None and log_every and iteration % log_every == 0:
                    logged.append((iteration, loss.detach()))
            iteration += 1
            nb += 1
            if max_steps and nb >= max_steps:
                break
        if logged:
            for (it, _), v in zip(logged, torch.stack([v for _, v in logged]).tolist()):
                writer.add_scalar("Loss/train_batch", v, it)
        running_loss = host_loss if reference_loop else float(loss_sum.item())
        dt = time.time() - t0
        acc = None
        if test_loader is not None and (reference_loop or (eval_iter and epoch % eval_iter == 0)):
            from sklearn.metrics import accuracy_score
            acc = round(float(evaluate(model, test_loader, accuracy_score)), 2)
            if writer is not None:
                writer.add_scalar("val?acc", acc, epoch)
        if rank == 0:
            os.makedirs(checkpoint_dir, exist_ok=True)
            torch.save({"epoch": epoch, "model_state_dict": model.state_dict(),
                        "optimizer_state_dict": optimizer.state_dict(), "loss": running_loss, "step": iteration},
                       os.path.join(checkpoint_dir, f"{epoch}.pt"))
            ips = nb * configs.batch_size * world / max(dt, 1e-9)
            print(f"Epoch {epoch}, curr loss: {running_loss:.4f}, mean_accuracy: {acc}, "
                  f"{nb} steps in {dt:.2f}s ({ips:.1f} img/s over {world} GPU(s))", flush=True)
    return running_loss


def time_steps(configs, steps, warmup, lr=1e-4, dev=None, seed=1234):
    """The hot loop body (train.py:91-98: forward, CE loss, zero_grad(set_to_none), backward, AdamW step) on one
    synthetic batch already resident on `dev`, dropout on; returns (seconds per timed step, last loss).  This is the
    repo's own CPU training step that bench.py's `cpu_baseline` times (BASELINE config 1)."""
    dev = torch.device(dev or device)
    torch.manual_seed(0)
    model = vit.VisionTransformer(configs).to(dev).train()
    opt = make_optimizer(model.parameters(), lr=lr, weight_decay=1e-4, device=dev)
    g = torch.Generator().manual_seed(seed)
    n_img = int(round((configs.num_patches ** 0.5) * configs.patch_size))
    x = torch.randn(configs.batch_size, configs.input_channels, n_img, n_img, generator=g).to(dev)
    y = torch.randint(0, configs.num_classes, (configs.batch_size,), generator=g).to(dev)
    loss = None
    t0 = time.perf_counter()
    for i in range(warmup + steps):
        if i == warmup:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
        loss = cross_entropy(model(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    last = float(loss.item())
    return (time.perf_counter() - t0) / max(steps, 1), last


def main():
    ap = argparse.ArgumentParser(description="ViT training on MI355X (drop-in for the reference src/train.py)")
    ap.add_argument("--model", default="tiny", choices=sorted(config.PRESETS))
    ap.add_argument("--img", type=int, default=64)
    ap.add_argument("--patch", type=int, default=16)
    ap.add_argument("--batch", type=int, default=8, help="per-GPU batch (CLS parameter is batch-shaped)")
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="max steps per epoch")
    ap.add_argument("--train-size", type=int, default=512)
    ap.add_argument("--test-size", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--eval-iter", type=int, default=1)
    ap.add_argument("--reference-loop", action="store_true",
                    help="the reference's loop bookkeeping exactly: validate every epoch, restart the step counter on "
                         "resume, host-summed loss (train.py:60-119)")
    ap.add_argument("--data", default="synthetic", choices=["synthetic", "synthetic-u8", "cifar10-bin", "folder"],
                    help="synthetic: N(0,1) float images at --img; the others decode uint8 images and apply the "
                         "reference transform (GPU kernel on cuda, Pillow on cpu)")
    ap.add_argument("--data-root", default=None)
    ap.add_argument("--checkpoint-dir", default="../checkpoints")
    ap.add_argument("--log-dir", default="../logs")
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"],
                    help="auto = cuda when a ROCm GPU is present, else cpu (train.py:26)")
    ap.add_argument("--threads", type=int, default=0, help="host-path threads (0 = every core this process may use)")
    ap.add_argument("--bench", action="store_true",
                    help="time --steps steps (after --warmup) on one resident synthetic batch; print one JSON line")
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    global device
    if args.device != "auto":
        device = args.device
    if device == "cpu":
        torch.set_num_threads(args.threads or len(os.sched_getaffinity(0)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        if device == "cuda":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    rank, world = _rank_world()
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    n_patches = (args.img // args.patch) ** 2
    D, H, L = config.PRESETS[args.model]
    cfg = config.ViTConfig(input_channels=3, num_classes=args.classes, num_patches=n_patches, embedding_size=D,
                           patch_size=args.patch, num_heads=H, num_blocks=L, precision=dtype,
                           batch_size=args.batch, device="cpu")
    if args.bench:
        steps = args.steps or 30
        sec, last = time_steps(cfg, steps, args.warmup, lr=args.lr)
        print(json.dumps({"device": device, "model": args.model, "img": args.img, "batch": args.batch,
                          "dtype": args.dtype, "threads": torch.get_num_threads(), "warmup": args.warmup,
                          "steps": steps, "ms_per_step": round(sec * 1e3, 3),
                          "images_per_s": round(args.batch / sec, 3), "final_loss": round(last, 5)}), flush=True)
        return
    pin = device == "cuda"
    if args.data == "synthetic":
        train_set = SyntheticImages(args.train_size, 3, args.img, args.classes, seed=1 + rank)
        test_set = SyntheticImages(args.test_size, 3, args.img, args.classes, seed=10_000)
    else:
        from VisionTransformer import data as D
        if args.data == "cifar10-bin":
            train_set, test_set = D.CIFAR10Bin(args.data_root, True), D.CIFAR10Bin(args.data_root, False)
        elif args.data == "folder":
            train_set = D.BrainTumorDataset(args.data_root, train=True, transform=D.decode)
            test_set = D.BrainTumorDataset(args.data_root, train=False, transform=D.decode)
        else:
            train_set = D.SyntheticRawImages(args.train_size, (32, 32, 3), args.classes, seed=1 + rank)
            test_set = D.SyntheticRawImages(args.test_size, (32, 32, 3), args.classes, seed=10_000)
    sampler = torch.utils.data.DistributedSampler(train_set) if world > 1 else None
    # the test set is sharded too (each sample on exactly one rank); evaluate() gathers the predictions
    tsampler = ShardSampler(test_set) if world > 1 else None
    if args.data != "synthetic" and device == "cuda":
        from VisionTransformer import data as D
        # one transform (and coefficient workspace) per loader: each stages its batches on its own side stream
        train_loader = D.DeviceBatches(D.raw_loader(train_set, args.batch, shuffle=True, num_workers=args.workers,
                                                    sampler=sampler), D.GpuImageTransform(args.img), device)
        test_loader = D.DeviceBatches(D.raw_loader(test_set, args.batch, shuffle=False, num_workers=args.workers,
                                                   drop_last=False, sampler=tsampler), D.GpuImageTransform(args.img),
                                      device)
    else:
        if args.data != "synthetic":
            from VisionTransformer import data as D
            train_set, test_set = (D.Transformed(s, D.host_transform(args.img)) for s in (train_set, test_set))
        train_loader = torch.utils.data.DataLoader(train_set, batch_size=args.batch, shuffle=sampler is None,
                                                   sampler=sampler, num_workers=args.workers, drop_last=True,
                                                   pin_memory=pin)
        # a partial last test batch is padded by evaluate() (the CLS parameter is batch-shaped)
        test_loader = torch.utils.data.DataLoader(test_set, batch_size=args.batch, num_workers=args.workers,
                                                  sampler=tsampler, drop_last=False, pin_memory=pin)
    train(cfg, train_loader, test_loader, args.epochs, args.eval_iter, args.log_dir, args.checkpoint_dir,
          lr=args.lr, max_steps=args.steps, reference_loop=args.reference_loop)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
