"""CPU-only checks of the drop-in package: module tree / init parity with the reference (golden sha256), the C-ABI
library exports every declared symbol (no compute calls), loud failure without a GPU, fused-layout bookkeeping,
and the data-parallel gradient bucketing under torch.distributed gloo (world size 2)."""
import json
import os
import re
import socket

import pytest
import torch

from oracle import vit_oracle as O
from VisionTransformer import _engine, _lib, config, transformer, vit

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(name):
    if name == "micro":
        return config.ViTConfig(3, 10, 4, 64, 16, 4, 2, "cpu", 4)
    return config.ViTConfig(3, 10, 16, 192, 16, 3, 12, "cpu", 8)


@pytest.mark.parametrize("name", ["micro", "tiny"])
def test_init_and_keys_match_reference(golden_dir, name):
    ref = json.load(open(os.path.join(golden_dir, "init_sha256.json")))
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg(name))
    sd = m.state_dict()
    assert list(sd.keys()) == ref[name + "_keys"]
    assert dict(O.state_sha256(sd)) == ref[name]


def test_state_dict_roundtrip_with_oracle_keys():
    cfg = _cfg("micro")
    torch.manual_seed(3)
    m = vit.VisionTransformer(cfg)
    st = O.init_state(O.make_config("micro", img=32, batch=4), seed=9)
    m.load_state_dict(st)
    for k, v in m.state_dict().items():
        assert torch.equal(v, st[k])


def test_host_path_matches_reference_goldens(golden_dir):
    """CPU model + CPU input runs the package's own host path (VisionTransformer/_cpu.py: fused QKV GEMM + batched
    attention with the multiplied sqrt(hd) scale), never the oracle: G1 micro logits / loss / every gradient."""
    import numpy as np
    g = np.load(os.path.join(golden_dir, "micro.npz"))
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg("micro")).eval()
    x, y = torch.from_numpy(g["x"]), torch.from_numpy(g["y"])
    logits = m(x)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    np.testing.assert_allclose(logits.detach().numpy(), g["logits"], atol=1e-5, rtol=0)
    assert abs(loss.item() - float(g["loss"])) < 1e-6
    for k, p in m.named_parameters():
        ref = g["grad/" + k]
        assert np.abs(p.grad.numpy() - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max()), k


def test_host_path_c1_and_module_api(golden_dir):
    """BASELINE config 1 dims (ViT-Tiny/16 64^2 B8) on the host path vs the reference's fp32 logits (G4), and the
    module-level API (Head returns (out, wei); MultiHeadAttention sets attention_probs) on CPU tensors."""
    import numpy as np
    g = np.load(os.path.join(golden_dir, "tiny.npz"))
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg("tiny")).eval()
    x, _ = O.synthetic_batch(O.make_config("tiny", img=64, batch=8))
    with torch.no_grad():
        logits = m(x)
    np.testing.assert_allclose(logits.numpy(), g["logits"], atol=2e-4, rtol=0)
    gk = np.load(os.path.join(golden_dir, "ops.npz"))
    head = transformer.Head(16, 64, 5)
    with torch.no_grad():
        head.query.weight.copy_(torch.from_numpy(gk["head/wq"]))
        head.key.weight.copy_(torch.from_numpy(gk["head/wk"]))
        head.value.weight.copy_(torch.from_numpy(gk["head/wv"]))
    out, wei = head(torch.from_numpy(gk["head/x"]))
    np.testing.assert_allclose(out.detach().numpy(), gk["head/out"], atol=1e-5)
    np.testing.assert_allclose(wei.numpy(), gk["head/wei"], atol=1e-6)
    mh = transformer.MultiHeadAttention(2, 8, 16, 5).eval()
    mh(torch.randn(3, 5, 16))
    assert tuple(mh.attention_probs.shape) == (3, 2, 5, 5)


def test_device_ops_refuse_host_tensors():
    """The HIP ops never compute on host tensors (no CPU fallback inside the device path)."""
    from VisionTransformer import _ops
    a = torch.zeros(4, 4)
    with pytest.raises(RuntimeError, match="ROCm device"):
        _ops.gemm(a, a, a, 4, 4, 4, 4, 4, 4)


def test_missing_library_raises(monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libvit_hip.so")
    with pytest.raises(_lib.HipLibraryError, match="no CPU fallback"):
        _lib.load()


def test_deepcopy_and_pickle_drop_the_engine():
    import copy
    import pickle
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg("micro"))
    eng = m.hip_engine
    eng._build(m, torch.device("cpu"))
    for clone in (copy.deepcopy(m), pickle.loads(pickle.dumps(m))):
        assert clone._engine is None and clone.hip_engine is not eng and clone.hip_engine.model_ref() is clone
        assert all(_engine.shadow_of(p) is None for p in clone.parameters())
        for (k, a), b in zip(m.state_dict().items(), clone.state_dict().values()):
            assert torch.equal(a, b) and a.data_ptr() != b.data_ptr(), k


def test_train_py_host_path_runs_c1_loop(tmp_path):
    """train.py --device cpu: the reference loop (train.py:89-102) with checkpoint + resume on the host path."""
    import subprocess
    import sys
    cmd = [sys.executable, os.path.join(ROOT, "vision-transformer_amd", "train.py"), "--device", "cpu", "--model",
           "tiny", "--img", "64", "--batch", "8", "--steps", "3", "--train-size", "32", "--test-size", "16",
           "--epochs", "1", "--workers", "0", "--threads", "2", "--checkpoint-dir", str(tmp_path / "ck"),
           "--log-dir", str(tmp_path / "logs")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sorted(os.listdir(tmp_path / "ck")) == ["0.pt", "1.pt"]
    ck = torch.load(tmp_path / "ck" / "1.pt", weights_only=True)
    assert ck["step"] == 6 and "transformer_encoder.blocks.11.multi_head.heads.2.query.weight" in ck["model_state_dict"]
    r = subprocess.run(cmd[:-4] + ["--bench", "--steps", "2", "--warmup", "1"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["device"] == "cpu" and line["steps"] == 2 and line["ms_per_step"] > 0


def test_train_reference_loop_bookkeeping(tmp_path, monkeypatch):
    """train(reference_loop=True): validation after EVERY epoch whatever eval_iter says (reference train.py:103,114),
    the step counter restarting at 0 on resume (:67) and the epoch loss summed on the host from loss.item() (:97-99);
    the default loop validates every eval_iter epochs and continues the step counter."""
    import train as T
    from VisionTransformer import config
    cfg = config.ViTConfig(3, 4, 4, 32, 16, 2, 1, "cpu", 4)
    monkeypatch.setattr(T, "device", "cpu")
    calls = []
    monkeypatch.setattr(T, "evaluate", lambda model, loader, metric: calls.append(1) or 0.5)
    ds = T.SyntheticImages(8, 3, 32, 4, seed=3)
    dl = torch.utils.data.DataLoader(ds, batch_size=4, drop_last=True)
    loss_ref = T.train(cfg, dl, dl, 2, 5, str(tmp_path / "l1"), str(tmp_path / "ck1"), reference_loop=True)
    assert len(calls) == 3                                  # epochs 0, 1, 2: every one
    assert torch.load(tmp_path / "ck1" / "2.pt", weights_only=True)["step"] == 6
    calls.clear()
    T.train(cfg, dl, dl, 3, 5, str(tmp_path / "l1"), str(tmp_path / "ck1"), reference_loop=True)   # resumes at 2
    assert torch.load(tmp_path / "ck1" / "3.pt", weights_only=True)["step"] == 4        # restarted at 0: 2 epochs
    calls.clear()
    T.train(cfg, dl, dl, 2, 5, str(tmp_path / "l2"), str(tmp_path / "ck2"))
    assert len(calls) == 1                                  # epoch 0 only (eval_iter 5)
    T.train(cfg, dl, dl, 3, 5, str(tmp_path / "l2"), str(tmp_path / "ck2"))
    assert torch.load(tmp_path / "ck2" / "3.pt", weights_only=True)["step"] == 10       # 6 + 2 epochs x 2 steps
    assert loss_ref > 0


def test_bench_spawns_ranks_dry_run():
    """`bench.py --gpus 2` without torchrun starts 2 ranks itself (spawn; the parent makes no GPU call) and rank 0
    prints one JSON line with n_gpus = 2, dp2, global batch 512 (the driver's --gpus N contract)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 512
    assert out["dry_run"] is True and out["value"] > 0
    assert "comm_exposed_ms" in out and out["comm_exposed_ms"] is not None and out["comm_exposed_ms"] >= 0
    assert out["grad_comm_dtype"] == "fp32"


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "vit_hip.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(vit_\w+)\s*\(", hdr, re.M))
    assert declared, "no declarations parsed"
    assert declared == set(_lib.EXPORTED_SYMBOLS), declared ^ set(_lib.EXPORTED_SYMBOLS)
    lib = _lib.load()                       # dlopen only; no kernel launches without a GPU
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.vit_abi_version() == _lib.ABI_VERSION


def test_host_abi_checker_c(tmp_path):
    """tests/host_abi_check.c, a plain-C host of the C-ABI (gcc, no GPU): version, options, error strings, the
    argument validation of the entry points and the host helpers.  tools/asan_host_check.sh runs the same program
    against an AddressSanitizer build of the library's host code (log: profiles/r3_asan_host_check.log)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    libdir = os.path.join(ROOT, "vision-transformer_amd", "VisionTransformer")
    exe = str(tmp_path / "host_abi_check")
    subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "host_abi_check.c"), "-o", exe, "-L", libdir, "-lvit_hip",
                    "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{libdir}", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout


def test_engine_roctx_ranges(monkeypatch):
    """engine.trace_ranges: every marked launch is bracketed by a roctx range named by its kernel family
    (torch.cuda.nvtx is roctx on ROCm; bench.py --roctx), balanced push / pop; off by default."""
    from VisionTransformer import _engine
    calls = []
    monkeypatch.setattr(torch.cuda.nvtx, "range_push", lambda name: calls.append(("push", name)))
    monkeypatch.setattr(torch.cuda.nvtx, "range_pop", lambda: calls.append(("pop", None)))
    eng = _engine.Engine.__new__(_engine.Engine)
    eng.profile_hook, eng.trace_ranges = None, False
    eng._mark("gemm_fwd", 0)
    eng._mark("gemm_fwd", 1)
    assert calls == []
    eng.trace_ranges = True
    for fam in ("gemm_fwd", "attn_bwd"):
        eng._mark(fam, 0, 1.0, 2.0)
        eng._mark(fam, 1)
    assert calls == [("push", "gemm_fwd"), ("pop", None), ("push", "attn_bwd"), ("pop", None)]


def test_library_options_host_only():
    """vit_set_option / vit_get_option (vit_hip.h): the documented names and shipped defaults, set/restore, and an
    unknown name refused — host-side only, and the library never reads the environment (no getenv in csrc/)."""
    defaults = {"gemm_impl": 0, "gemm_tail": 0, "gemm_tail_min_kt": 40, "splitk_min_kt": 0, "gemm_group_m": 0,
                "gemm_epi_general": 0, "gemm_persist": 1, "attn_fwd_split": 0, "attn_bwd_split": 0,
                "attn_bwd_grid": 0, "ln16": 1, "ln_al": 1, "attn_fwd_ring": 1, "gemm_tail_v2": 0,
                "splitk_rounds": 1, "attn_fwd_grid": 0}
    for k, v in defaults.items():
        assert _lib.get_option(k) == v, k
    with _lib.option("gemm_persist", 0):
        assert _lib.get_option("gemm_persist") == 0
    assert _lib.get_option("gemm_persist") == 1
    with pytest.raises(RuntimeError):
        _lib.set_option("no_such_option", 1)
    with pytest.raises(KeyError):
        _lib.get_option("no_such_option")
    csrc = os.path.join(ROOT, "vision-transformer_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h")):
            assert "getenv" not in open(os.path.join(csrc, f)).read(), f


def test_dropout_seed_twins():
    for base in (0, 1, 12345, 2 ** 31 - 2):
        for l in range(3):
            for s in range(2):
                assert _engine.site_seed(base, l, s) == O.site_seed(base, l, s)
    import numpy as np
    idx = np.arange(1000, dtype=np.uint64)
    ref = O.hash_u32(777, idx)
    assert all(int(ref[i]) == _engine._hash_u32(777, i) for i in range(0, 1000, 37))


def test_engine_layout_views():
    """Per-head grads are views of the fused QKV gradient rows: q heads, then k heads, then v heads."""
    torch.manual_seed(0)
    cfg = _cfg("micro")
    m = vit.VisionTransformer(cfg)
    eng = m.hip_engine
    eng._build(m, torch.device("cpu"))
    D, hd = 64, 16
    for l in range(2):
        fused = eng.gw[f"{l}.qkv_w"]
        for h in range(4):
            head = m.transformer_encoder.blocks[l].multi_head.heads[h]
            gv = dict((id(p), g) for p, g in eng.grad_views)
            assert gv[id(head.query.weight)].data_ptr() == fused[h * hd].data_ptr()
            assert gv[id(head.key.weight)].data_ptr() == fused[D + h * hd].data_ptr()
            assert gv[id(head.value.weight)].data_ptr() == fused[2 * D + h * hd].data_ptr()
            assert _engine.shadow_of(head.query.weight).data_ptr() == eng.ww[f"{l}.qkv_w"][h * hd].data_ptr()
    # buckets: head | block L-1 | ... | block 0 | embedding, contiguous and ordered
    rngs = [eng.head_range] + [eng.block_range[l] for l in reversed(range(2))] + [eng.embed_range]
    for (a0, b0), (a1, b1) in zip(rngs, rngs[1:]):
        assert b0 == a1
    assert rngs[-1][1] == eng.G.numel()
    # every parameter gets a gradient view of its own shape, all disjoint
    spans = sorted((g.data_ptr(), g.data_ptr() + 4 * g.numel()) for _, g in eng.grad_views)
    for (s0, e0), (s1, e1) in zip(spans, spans[1:]):
        assert e0 <= s1
    assert all(g.shape == p.shape for p, g in eng.grad_views)
    assert len(eng.grad_views) == len(list(m.parameters()))


def test_attach_grads_semantics():
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg("micro"))
    eng = m.hip_engine
    eng._build(m, torch.device("cpu"))
    assert eng._attach_grads() == 0.0          # all None -> overwrite; the views are attached at backward's end
    assert all(p.grad is None for p in m.parameters())
    eng._attach_pending()
    assert all(p.grad is not None for p in m.parameters())
    assert eng._attach_grads() == 1.0          # live views -> accumulate (zero_grad(set_to_none=False) style)
    p0 = next(m.parameters())
    p0.grad = None
    eng.G.fill_(3.0)
    assert eng._attach_grads() == 1.0          # mixed -> the dropped one is zeroed, others accumulate
    assert torch.all(p0.grad == 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ddp_worker(rank, world, port, q, comm_dtype=torch.float32):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg("micro"))
    eng = m.hip_engine
    eng._build(m, torch.device("cpu"))
    eng.ddp_enabled = True
    eng.comm_dtype = comm_dtype
    # rank-dependent values that are not bf16-exact, so the bf16 path's rounding is visible
    base = torch.arange(eng.G.numel(), dtype=torch.float32) / 7.0 + 0.001
    eng.G.copy_(base * (rank + 1))
    for rng in [eng.head_range] + [eng.block_range[l] for l in reversed(range(2))] + [eng.embed_range]:
        eng._bucket_ready(rng)
    eng._finish_buckets()
    ranks = [base * (r + 1) for r in range(world)]
    if comm_dtype == torch.bfloat16:
        # each rank's gradients rounded to bf16, summed in bf16 (gloo), widened and averaged
        acc = ranks[0].bfloat16()
        for g in ranks[1:]:
            acc = acc + g.bfloat16()
        expect = acc.float() * (1.0 / world)
        ok = torch.equal(eng.G, expect)
    else:
        ok = torch.allclose(eng.G, sum(ranks) / world)
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def _launch_mode_worker(port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    m = vit.VisionTransformer(_cfg("micro"))
    out = {}
    for mode in ("auto", "shared", "persistent"):
        out[mode] = m.enable_data_parallel(force=True, launch_mode=mode).hip_engine.shared_cus
    try:
        m.enable_data_parallel(force=True, launch_mode="bogus")
        out["bad"] = "accepted"
    except ValueError:
        out["bad"] = "refused"
    q.put(out)
    dist.destroy_process_group()


def test_enable_data_parallel_launch_mode():
    """enable_data_parallel(launch_mode=...): 'auto' keeps the persistent grids (the CU-hog A/B),
    'shared' / 'persistent' force a mode (bench.py --launch-mode); anything else is refused."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_launch_mode_worker, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=120)
    p.join(timeout=60)
    assert out == {"auto": False, "shared": True, "persistent": False, "bad": "refused"}


@pytest.mark.parametrize("comm_dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_ddp_gradient_buckets_gloo(comm_dtype):
    """2-rank gloo: every bucket of the flat gradient buffer is averaged across ranks; with bf16 buckets
    (enable_data_parallel(grad_dtype=torch.bfloat16)) the result is exactly the average of the bf16-rounded
    gradients."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q, comm_dtype)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


class _IndexedImages(torch.utils.data.Dataset):
    """Synthetic images that record which indices were read (shard order per epoch)."""

    def __init__(self, n):
        import train as T
        self.base = T.SyntheticImages(n, 3, 32, 4, seed=3)
        self.seen = []

    def __len__(self):
        return len(self.base)

    def __getitem__(self, i):
        self.seen.append(int(i))
        return self.base[i]


class _SignClassifier(torch.nn.Module):
    """Predicts (number of positive pixels) mod 4: a deterministic stand-in whose accuracy is known exactly."""

    def forward(self, x):
        k = (x > 0).flatten(1).sum(1) % 4
        return torch.nn.functional.one_hot(k, 4).float()


def _dp_train_worker(rank, world, port, q):
    import torch.distributed as dist
    import train as T
    from VisionTransformer import config
    from sklearn.metrics import accuracy_score
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    T.device = "cpu"
    ds = _IndexedImages(16)
    sampler = torch.utils.data.DistributedSampler(ds, seed=0)
    dl = torch.utils.data.DataLoader(ds, batch_size=4, sampler=sampler, drop_last=True)
    cfg = config.ViTConfig(3, 4, 4, 32, 16, 2, 1, "cpu", 4)
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        T.train(cfg, dl, None, 1, 1, os.path.join(tmp, "l"), os.path.join(tmp, "ck"))     # epochs 0 and 1
    orders = [ds.seen[:8], ds.seen[8:16]]
    # after train() each replica's CPU RNG (the host dropout's) is its own stream: keep masks differ per rank
    drop = torch.nn.functional.dropout(torch.ones(256), 0.2, True).ne(0).tolist()
    # evaluate(): each rank scores its shard of a test set whose size (37) divides neither by the world size nor by the
    # batch: ShardSampler shards (partial last batches, padded for the model), and DistributedSampler shards (padding
    # duplicates dropped); both must give the accuracy over the 37 unique samples
    ts = T.SyntheticImages(37, 3, 32, 4, seed=7)
    x, y = next(iter(torch.utils.data.DataLoader(ts, batch_size=37)))
    want = float((_SignClassifier()(x).argmax(-1) == y).double().mean())
    accs = []
    for smp in (T.ShardSampler(ts), torch.utils.data.DistributedSampler(ts, shuffle=False),
                torch.utils.data.DistributedSampler(ts, shuffle=True, seed=3)):
        tl = torch.utils.data.DataLoader(ts, batch_size=4, drop_last=False, sampler=smp)
        accs.append(T.evaluate(_SignClassifier(), tl, accuracy_score))
    # a ViT with a batch-shaped CLS parameter: each rank's partial last batch (rank 0: 19 = 4 x 4 + 3, rank 1: 18 =
    # 4 x 4 + 2 samples) is padded for the forward and only its real rows are scored.  The CLS row differs per batch
    # position, so the expected value replays each rank's batches.
    from VisionTransformer import vit as V
    torch.manual_seed(0)
    vm = V.VisionTransformer(config.ViTConfig(3, 4, 4, 32, 16, 2, 1, "cpu", 4))
    tl = torch.utils.data.DataLoader(ts, batch_size=4, drop_last=False, sampler=T.ShardSampler(ts))
    v_acc = T.evaluate(vm, tl, accuracy_score)
    correct = 0
    with torch.no_grad():
        vm.eval()
        for r in range(world):
            idx = list(range(r, 37, world))
            xs, ys = x[idx], y[idx]
            pad = (-len(idx)) % 4
            xp = torch.cat([xs, xs[-1:].expand(pad, 3, 32, 32)])
            pr = torch.cat([vm(xp[i:i + 4]) for i in range(0, len(xp), 4)])[:len(idx)].argmax(-1)
            correct += int((pr == ys).sum())
    v_want = correct / 37
    q.put((rank, orders, accs, want, v_acc, v_want, drop))
    dist.destroy_process_group()


def test_data_parallel_train_epochs_and_evaluate_gloo():
    """2-rank gloo, host path: train() calls DistributedSampler.set_epoch every epoch,
    so each rank's shard order differs between epochs and the two ranks' shards partition the set; evaluate() on a
    sharded test loader returns the accuracy over the WHOLE test set on every rank, each sample counted once, also
    when the set divides neither by the world size nor by the batch."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    (r0, o0, a0, w0, v0, vw0, d0), (r1, o1, a1, w1, v1, vw1, d1) = res
    assert d0 != d1                                               # per-replica dropout streams
    for e in range(2):
        assert sorted(o0[e] + o1[e]) == list(range(16)), e       # the shards partition the set every epoch
    assert o0[0] != o0[1] and o1[0] != o1[1]                      # set_epoch: a new order each epoch
    assert 0.0 < w0 < 1.0 and w0 == w1
    for a in a0 + a1:
        assert abs(a - w0) < 1e-12, (a0, a1, w0)                  # exact whole-set accuracy over unique samples
    assert abs(v0 - vw0) < 1e-12 and v0 == v1


def _dropout_rank_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = vit.VisionTransformer(_cfg("micro")).enable_data_parallel()
    q.put((rank, m.hip_engine.dropout_rank))
    dist.destroy_process_group()


def test_data_parallel_dropout_differs_per_rank():
    """Every rank draws the same base dropout seed (identically seeded CPU RNG, needed for identical init), so the
    engine folds the replica index in: enable_data_parallel sets it to the group rank; rank 0 keeps
    the single-process seed; the ranks' seeds, and the keep masks they hash to at every site, all differ."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dropout_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == [(0, 0), (1, 1)]
    for base in (0, 1, 12345, 2 ** 31 - 2):
        seeds = [_engine.dropout_seed(base, r) for r in range(8)]
        assert seeds[0] == base and len(set(seeds)) == 8 and all(0 <= s < 2 ** 31 for s in seeds)
        for layer in (0, 11):
            for site in (0, 1):
                masks = [O.dropout_keep(_engine.site_seed(s, layer, site), (197, 64)) for s in seeds]
                for i in range(8):
                    assert abs(masks[i].float().mean().item() - 0.8) < 0.02
                    for j in range(i):
                        assert not torch.equal(masks[i], masks[j])


def test_attention_probs_warns_once_after_fused_forward():
    """The fused forward keeps attention probabilities only with store_attention_probs=True; reading them after a
    forward that skipped them returns None (as before) but warns once, pointing at the flag."""
    import warnings
    mh = transformer.MultiHeadAttention(2, 8, 16, 5)
    assert mh.attention_probs is None                     # never ran: no warning
    transformer._PROBS_WARNED = False
    mh.attention_probs = None
    mh._probs_skipped = True                              # what the engine records after a fused forward
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert mh.attention_probs is None
        assert mh.attention_probs is None
    assert len(w) == 1 and "store_attention_probs" in str(w[0].message)
    mh.attention_probs = torch.zeros(1)                   # module-level forward stores them: no warning path
    assert mh.attention_probs is not None and not mh._probs_skipped


def test_attention_probs_auto_rule_and_host_path(golden_dir, probs_auto_budget):
    """store_attention_probs=None (the default): attention_probs are filled on every forward whose probabilities fit
    in vit.ATTENTION_PROBS_AUTO_BYTES (the reference fills them always, transformer.py:48) — C1 (ViT-Tiny 64^2 B8)
    and ViT-B/16 224^2 up to 12 images, not the C2 batch of 256; True / False override.  The host path with them on
    still matches the reference's C1 logits (G4)."""
    import types
    import numpy as np
    base = config.ViTConfig.preset("base", img_size=224, batch_size=256, device="cpu")
    fake = types.SimpleNamespace(store_attention_probs=None, vit_config=base)
    per_image = base.num_heads * (base.num_patches + 1) ** 2 * 4 * base.num_blocks
    bmax = probs_auto_budget // per_image
    assert bmax == 12
    wants = lambda b: vit.VisionTransformer.wants_attention_probs(fake, b)      # noqa: E731
    assert wants(1) and wants(bmax) and not wants(bmax + 1) and not wants(256)
    fake.store_attention_probs = True
    assert wants(256)
    fake.store_attention_probs = False
    assert not wants(1)
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg("tiny")).eval()
    assert m.store_attention_probs is None and m.wants_attention_probs(8)
    g = np.load(os.path.join(golden_dir, "tiny.npz"))
    x, _ = O.synthetic_batch(O.make_config("tiny", img=64, batch=8))
    with torch.no_grad():
        logits = m(x)
    np.testing.assert_allclose(logits.numpy(), g["logits"], atol=2e-4, rtol=0)
    for blk in m.transformer_encoder.blocks:
        p = blk.multi_head.attention_probs
        assert p is not None and tuple(p.shape) == (8, 3, 17, 17)
        torch.testing.assert_close(p.sum(-1), torch.ones(8, 3, 17), atol=1e-5, rtol=0)
    m.store_attention_probs = False
    with torch.no_grad():
        m(x)
    assert all(b.multi_head.attention_probs is None for b in m.transformer_encoder.blocks)
