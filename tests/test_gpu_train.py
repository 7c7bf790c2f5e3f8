"""GPU tests of the training entry points: data-parallel gradient averaging through the engine's bucketed all-reduce
(two ranks sharing the one GPU of the test box, gloo transport — the 8-GPU RCCL run is the driver's scaling bench),
and train.py's loop / checkpoint / resume contract (train.py:52-58,63-78,107-113)."""
import os
import socket
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    from VisionTransformer import config
    return config.ViTConfig(3, 10, 16, 128, 16, 2, 2, "cpu", 4)      # hd = 64, 64x64 images, B = 4 per rank


def _batch(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(4, 3, 64, 64, generator=g), torch.randint(0, 10, (4,), generator=g)


def _ddp_worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-transformer_amd")]
    import torch.distributed as dist
    from VisionTransformer import vit
    from VisionTransformer.optim import FusedAdamW, cross_entropy
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg()).cuda().eval().enable_data_parallel()
    opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    x, y = _batch(rank)
    for _ in range(2):
        loss = cross_entropy(m(x.cuda()), y.cuda())
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    if rank == 0:
        q.put({k: v.detach().cpu().numpy() for k, v in m.state_dict().items()})   # by value, not shared fds
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_equals_gradient_accumulation():
    """2-rank DDP step == one process averaging the two ranks' gradients (SURVEY.md §8e parity check)."""
    import torch.multiprocessing as mp
    from VisionTransformer import vit
    from VisionTransformer.optim import FusedAdamW, cross_entropy
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ddp_state = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg()).cuda().eval()
    opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    for _ in range(2):
        acc = None
        for r in range(2):
            x, y = _batch(r)
            loss = cross_entropy(m(x.cuda()), y.cuda())
            for p in m.parameters():
                p.grad = None
            loss.backward()
            g = m.hip_engine.G.clone()
            acc = g if acc is None else acc + g
        m.hip_engine.G.copy_(acc / 2)
        opt.step()
    for k, v in m.state_dict().items():
        assert (v.cpu() - torch.from_numpy(ddp_state[k])).abs().max().item() < 1e-5, k


def _keep_bits(m, x, seed):
    """proj-dropout keep bits (VIT_MASK4 bytes) of block 0 in one training forward drawn under CPU seed `seed`."""
    torch.manual_seed(seed)
    _, tape = m.hip_engine.forward(x, True, save=True)
    return tape.blocks[0][14].cpu().numpy()


def _ddp_train_worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-transformer_amd")]
    import torch.distributed as dist
    from VisionTransformer import vit
    from VisionTransformer.optim import FusedAdamW, cross_entropy
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg()).cuda().train().enable_data_parallel()
    opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    x, y = _batch(rank)
    for _ in range(2):
        loss = cross_entropy(m(x.cuda()), y.cuda())
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()} if rank == 0 else None
    q.put((rank, m.hip_engine.dropout_rank, state, _keep_bits(m, x.cuda(), 7)))
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_train_mode_equals_per_rank_accumulation():
    """Train mode, dropout on: a 2-rank data-parallel step equals one process that
    accumulates the two ranks' micro-batches, each drawn under that rank's dropout stream (the same CPU RNG state,
    the rank folded into the seed), within 1e-5 after two AdamW steps; and the two ranks' keep bits differ (before the
    fix every replica applied the same masks)."""
    import numpy as np
    import torch.multiprocessing as mp
    from VisionTransformer import vit
    from VisionTransformer.optim import FusedAdamW, cross_entropy
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [0, 1]
    ddp_state = res[0][2]
    assert not np.array_equal(res[0][3], res[1][3])              # replicas draw different keep bits
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg()).cuda().train()
    opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    eng = m.hip_engine
    for _ in range(2):
        st = torch.get_rng_state()          # every rank draws its base seed from the same CPU RNG state
        acc = None
        for r in range(2):
            torch.set_rng_state(st)
            eng.dropout_rank = r
            x, y = _batch(r)
            loss = cross_entropy(m(x.cuda()), y.cuda())
            for p in m.parameters():
                p.grad = None
            loss.backward()
            g = eng.G.clone()
            acc = g if acc is None else acc + g
        eng.G.copy_(acc / 2)
        opt.step()
    for k, v in m.state_dict().items():
        assert (v.cpu() - torch.from_numpy(ddp_state[k])).abs().max().item() < 1e-5, k
    for r in range(2):                      # the single process reproduces each rank's masks exactly
        eng.dropout_rank = r
        assert np.array_equal(_keep_bits(m, _batch(r)[0].cuda(), 7), res[r][3]), r


def test_train_loop_checkpoint_and_resume(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
    import train as T
    from VisionTransformer import config
    cfg = config.ViTConfig(3, 10, 16, 128, 16, 2, 2, "cpu", 4, precision=torch.bfloat16)
    ds = T.SyntheticImages(32, 3, 64, 10, seed=3)
    loader = torch.utils.data.DataLoader(ds, batch_size=4, drop_last=True)
    ck, logs = str(tmp_path / "ck"), str(tmp_path / "logs")
    l0 = T.train(cfg, loader, loader, epochs=1, eval_iter=1, log_dir=logs, checkpoint_dir=ck, lr=1e-3)
    assert sorted(os.listdir(ck)) == ["0.pt", "1.pt"] and T.search_checkpoint(ck) == 1
    ckpt = torch.load(os.path.join(ck, "1.pt"), weights_only=True)
    assert set(ckpt) == {"epoch", "model_state_dict", "optimizer_state_dict", "loss", "step"}
    assert "transformer_encoder.blocks.0.multi_head.heads.1.value.weight" in ckpt["model_state_dict"]
    assert ckpt["step"] == 16 and abs(ckpt["loss"] - l0) < 1e-6
    # resume: picks up epoch 1, re-runs it (reference semantics: range(saved_epoch, epochs + 1))
    l1 = T.train(cfg, loader, loader, epochs=1, eval_iter=1, log_dir=logs, checkpoint_dir=ck, lr=1e-3)
    ck2 = torch.load(os.path.join(ck, "1.pt"), weights_only=True)
    assert ck2["step"] == 24 and torch.isfinite(torch.tensor(l1))
