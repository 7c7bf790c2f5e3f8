"""Pin the oracle (oracle/vit_oracle.py) against golden vectors produced by the reference itself
(tests/golden/gen_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import vit_oracle as O


def _npz(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


@pytest.mark.parametrize("name,kw", [("micro", dict(model="micro", img=32, batch=4)),
                                     ("tiny", dict(model="tiny", img=64, batch=8))])
def test_init_bit_exact(golden_dir, name, kw):
    """G0: oracle init reproduces the reference state_dict (keys, order, every bit) under manual_seed(0)."""
    ref = json.load(open(os.path.join(golden_dir, "init_sha256.json")))
    cfg = O.make_config(**kw)
    st = O.init_state(cfg, seed=0)
    assert list(st.keys()) == ref[name + "_keys"]
    got = O.state_sha256(st)
    assert dict(got) == ref[name]


def test_micro_logits_loss_grads(golden_dir):
    """G1: eval-mode logits, CE loss and every parameter gradient vs the reference (fp32)."""
    g = _npz(golden_dir, "micro.npz")
    cfg = O.make_config("micro", img=32, batch=4)
    st = O.init_state(cfg, 0)
    x, y = torch.from_numpy(g["x"]), torch.from_numpy(g["y"])
    logits, loss, grads = O.loss_and_grads(st, x, y, cfg)
    np.testing.assert_allclose(logits.numpy(), g["logits"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(float(loss), float(g["loss"]), rtol=1e-6, atol=1e-6)
    for k, v in grads.items():
        ref = g["grad/" + k]
        scale = max(1.0, float(np.abs(ref).max()))
        np.testing.assert_allclose(v.numpy(), ref, rtol=0, atol=2e-5 * scale, err_msg=k)


def test_synthetic_batch_matches_golden_inputs(golden_dir):
    g = _npz(golden_dir, "micro.npz")
    cfg = O.make_config("micro", img=32, batch=4)
    x, y = O.synthetic_batch(cfg)
    assert np.array_equal(x.numpy(), g["x"]) and np.array_equal(y.numpy(), g["y"])


def test_tiny_c1(golden_dir):
    """G4: ViT-Tiny/16 64^2 B8 (BASELINE config 1): logits, loss, grad norms, 3-step AdamW trace."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = _npz(golden_dir, "tiny.npz")
    cfg = O.make_config("tiny", img=64, batch=8)
    st = O.init_state(cfg, 0)
    x, y = O.synthetic_batch(cfg)
    logits, loss, grads = O.loss_and_grads(st, x, y, cfg)
    np.testing.assert_allclose(logits.numpy(), g["logits"], rtol=0, atol=5e-4)
    np.testing.assert_allclose(float(loss), float(g["loss"]), rtol=1e-5)
    for k, n in zip(g["gnorm_keys"], g["gnorm"]):
        assert abs(float(grads[str(k)].double().norm()) - n) <= 5e-3 * max(n, 1e-3), k
    losses, st2 = O.train_steps(st, x, y, cfg, steps=3)
    np.testing.assert_allclose(losses, g["trace"], rtol=2e-5)
    for k, n in zip(g["post_keys"], g["post_norm"]):
        assert abs(float(st2[str(k)].double().norm()) - n) <= 1e-5 * max(n, 1.0), k


def test_ops_kats(golden_dir):
    """G3: per-op known answers from the reference modules."""
    g = _npz(golden_dir, "ops.npz")
    t = lambda k: torch.from_numpy(g[k])
    x = t("head/x").requires_grad_(True)
    out, wei = O.head_attention(x, t("head/wq"), t("head/wk"), t("head/wv"))
    np.testing.assert_allclose(out.detach().numpy(), g["head/out"], atol=1e-5)
    np.testing.assert_allclose(wei.detach().numpy(), g["head/wei"], atol=1e-6)
    out.backward(t("head/gout"))
    np.testing.assert_allclose(x.grad.numpy(), g["head/dx"], atol=1e-4)
    xl = t("ln/x").requires_grad_(True)
    w, b = t("ln/w").requires_grad_(True), t("ln/b").requires_grad_(True)
    yl = O.layer_norm(xl, w, b)
    np.testing.assert_allclose(yl.detach().numpy(), g["ln/y"], atol=1e-5)
    yl.backward(t("ln/gy"))
    np.testing.assert_allclose(xl.grad.numpy(), g["ln/dx"], atol=1e-5)
    np.testing.assert_allclose(w.grad.numpy(), g["ln/dw"], atol=1e-5)
    np.testing.assert_allclose(b.grad.numpy(), g["ln/db"], atol=1e-5)
    xf = t("ffn/x")
    yf = torch.relu(xf @ t("ffn/w1").t() + t("ffn/b1")) @ t("ffn/w2").t() + t("ffn/b2")
    np.testing.assert_allclose(yf.numpy(), g["ffn/y"], atol=1e-5)
    ce = torch.nn.functional.cross_entropy(t("ce/logits"), t("ce/labels"))
    np.testing.assert_allclose(float(ce), float(g["ce/loss"]), rtol=1e-6)
    # reference dropout is p=0.2 with 1/(1-p) scaling; the counter-hash masks must have the same statistics
    assert abs(float(g["dropout/zero_frac"]) - 0.2) < 0.01
    assert abs(float(g["dropout/nonzero_value"]) - 1.25) < 1e-6
    keep = O.dropout_keep(12345, (200000,))
    assert abs(1.0 - float(keep.float().mean()) - 0.2) < 0.005


def test_block_base_width(golden_dir):
    """G2: one ViT-B-width block (D768 H12 T197 B2) — the oracle's block equals the reference block."""
    g = _npz(golden_dir, "block_base.npz")
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    torch.manual_seed(11)
    # Block draw order: heads (key, query, value) x12, proj, fc1, fc2 (transformer.py:67-72)
    D, H = 768, 12
    hd = D // H
    p = {}
    for h in range(H):
        for nm in ("key", "query", "value"):
            p[f"{h}.{nm}"] = O._kaiming_linear(hd, D, bias=False)[0]
    p["proj.w"], p["proj.b"] = O._kaiming_linear(D, D)
    p["fc1.w"], p["fc1.b"] = O._kaiming_linear(4 * D, D)
    p["fc2.w"], p["fc2.b"] = O._kaiming_linear(D, 4 * D)
    for dt, tag, tol in ((torch.float32, "f32", 1e-5), (torch.float64, "f64", 1e-10)):
        P = {k: v.to(dt) for k, v in p.items()}
        xb = torch.randn(2, 197, D, generator=torch.Generator().manual_seed(12), dtype=torch.float64).to(dt)
        xb.requires_grad_(True)
        a = O.layer_norm(xb, torch.ones(D, dtype=dt), torch.zeros(D, dtype=dt))
        outs = [O.head_attention(a, P[f"{h}.query"], P[f"{h}.key"], P[f"{h}.value"])[0] for h in range(H)]
        e = xb + torch.cat(outs, -1) @ P["proj.w"].t() + P["proj.b"]
        a2 = O.layer_norm(e, torch.ones(D, dtype=dt), torch.zeros(D, dtype=dt))
        yb = e + torch.relu(a2 @ P["fc1.w"].t() + P["fc1.b"]) @ P["fc2.w"].t() + P["fc2.b"]
        gy = torch.randn(2, 197, D, generator=torch.Generator().manual_seed(13), dtype=torch.float64).to(dt)
        yb.backward(gy)
        np.testing.assert_allclose(yb.detach().double().reshape(-1)[::101].numpy(), g[f"{tag}/y_slice"],
                                   atol=tol * 10, rtol=tol)
        np.testing.assert_allclose(xb.grad.double().reshape(-1)[::101].numpy(), g[f"{tag}/dx_slice"],
                                   atol=tol * 100, rtol=tol * 10)


def test_notebook_sdpa_kat(golden_dir):
    """G5: the reference's only hand KAT (tests/multihead-attention-test.ipynb), divide-by-sqrt(d) variant."""
    k = json.load(open(os.path.join(golden_dir, "sdpa_notebook.json")))
    emb = torch.tensor(k["embeddings"])
    w = torch.tensor(k["qkv_weights"]).view(2, 2, 4, 6)
    Q, K, V = emb @ w[..., 0:2], emb @ w[..., 2:4], emb @ w[..., 4:6]
    s = torch.softmax(Q @ K.transpose(-2, -1) / 2 ** 0.5, -1)
    np.testing.assert_allclose((s @ V).numpy(), np.array(k["expected_out"]), atol=6e-4)


def test_seq_chain_variant_is_the_same_function(golden_dir):
    """The summation-order variant used for tolerance scales computes the same model (micro goldens, fp32)."""
    g = _npz(golden_dir, "micro.npz")
    cfg = O.make_config("micro", img=32, batch=4)
    st = O.init_state(cfg, 0)
    logits, loss, grads = O.loss_and_grads(st, torch.from_numpy(g["x"]), torch.from_numpy(g["y"]), cfg,
                                           seq_chain=True)
    np.testing.assert_allclose(logits.numpy(), g["logits"], atol=5e-5)
    for k, v in grads.items():
        ref = g["grad/" + k]
        np.testing.assert_allclose(v.numpy(), ref, atol=1e-4 * max(1.0, float(np.abs(ref).max())), err_msg=k)


def test_item_bh_split_exact_below_2_24():
    """csrc/vit_common.h item_bh(): the persistent attention kernels split item u = b * H + h with a float reciprocal
    and one correction step instead of a 64-bit division.  Emulated here with IEEE float32 (numpy) for every
    u < 2^24 — the bound the launchers enforce (vit_attention.hip) — and every head count 1..64."""
    import numpy as np
    u = np.arange(1 << 24, dtype=np.int64)
    uf = u.astype(np.float32)
    for hh in range(1, 65):
        q = (uf * (np.float32(1.0) / np.float32(hh))).astype(np.int64)      # float -> int truncates, as (int)
        r = u - q * hh
        lo, hi = r < 0, r >= hh
        q = q - lo + hi
        r = r + lo * hh - hi * hh
        assert np.array_equal(q, u // hh) and np.array_equal(r, u % hh), hh
