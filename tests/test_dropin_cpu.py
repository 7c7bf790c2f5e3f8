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


def test_cpu_forward_fails_loudly():
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg("micro"))
    with pytest.raises(RuntimeError, match="ROCm device"):
        m(torch.randn(4, 3, 32, 32))
    blk = m.transformer_encoder.blocks[0]
    with pytest.raises(RuntimeError, match="ROCm device"):
        blk(torch.randn(4, 5, 64))


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "vit_hip.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(vit_\w+)\s*\(", hdr, re.M))
    assert declared, "no declarations parsed"
    assert declared == set(_lib.EXPORTED_SYMBOLS), declared ^ set(_lib.EXPORTED_SYMBOLS)
    lib = _lib.load()                       # dlopen only; no kernel launches without a GPU
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.vit_abi_version() == _lib.ABI_VERSION


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
            assert head.query.weight._vit_shadow.data_ptr() == eng.ww[f"{l}.qkv_w"][h * hd].data_ptr()
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
    assert eng._attach_grads() == 0.0          # all None -> overwrite
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


def _ddp_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = vit.VisionTransformer(_cfg("micro"))
    eng = m.hip_engine
    eng._build(m, torch.device("cpu"))
    eng.ddp_enabled = True
    eng.G.copy_(torch.arange(eng.G.numel(), dtype=torch.float32) * (rank + 1))
    for rng in [eng.head_range] + [eng.block_range[l] for l in reversed(range(2))] + [eng.embed_range]:
        eng._bucket_ready(rng)
    eng._finish_buckets()
    expect = torch.arange(eng.G.numel(), dtype=torch.float32) * (sum(range(1, world + 1)) / world)
    q.put((rank, bool(torch.allclose(eng.G, expect))))
    dist.destroy_process_group()


def test_ddp_gradient_buckets_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]
