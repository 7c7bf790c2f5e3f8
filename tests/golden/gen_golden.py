"""Generate golden vectors by importing the REFERENCE model (build container only; /root/reference is read-only and
absent on the GPU box).  Run:  python tests/golden/gen_golden.py

Outputs (small, committed):
  G0  init_sha256.json      sha256 of every reference state_dict tensor after torch.manual_seed(0) (micro, tiny)
  G1  micro.npz             micro config: input, eval logits, CE loss, all grads (eval mode: dropout off)
  G3  ops.npz               per-op KATs: Head (x sqrt(hd)), LayerNorm fwd/bwd, FeedForward, classifier MLP, CE
  G4  tiny.npz              C1 (ViT-Tiny/16, 64^2, B8): eval logits, loss, grad norms, 3-step AdamW loss trace
  G2  block_base.npz        one ViT-B-width Block (D768 H12 T197 B2): fp32/fp64 output + dx summaries
  G5  sdpa_notebook.json    tests/multihead-attention-test.ipynb known-answer values (÷sqrt(d) variant)

Nothing from the reference's source is stored: only inputs/outputs (data).
"""
import hashlib
import json
import math
import os
import sys

sys.dont_write_bytecode = True
REF = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))

import numpy as np
import torch

sys.path.insert(0, REF)
from VisionTransformer import config as rconfig, transformer as rtransformer, vit as rvit  # noqa: E402

torch.set_num_threads(8)


def sha(t):
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()


def ref_model(D, H, L, img, B, nc, C=3, P=16, seed=0):
    n = (img // P) ** 2
    cfg = rconfig.ViTConfig(input_channels=C, num_classes=nc, num_patches=n, embedding_size=D, patch_size=P,
                            num_heads=H, num_blocks=L, device="cpu", batch_size=B)
    torch.manual_seed(seed)
    return rvit.VisionTransformer(cfg), cfg


def batch(B, C, img, nc, seed=1234):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, C, img, img, generator=g)
    g2 = torch.Generator().manual_seed(seed + 1)
    y = torch.randint(0, nc, (B,), generator=g2)
    return x, y


def run_eval_grads(model, x, y):
    model.eval()                               # dropout off -> deterministic; autograd still records
    model.zero_grad(set_to_none=True)
    logits = model(x)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    return logits.detach(), loss.detach(), grads


def main():
    out = {}
    # ---------------- G0 + G1: micro ----------------
    specs = {"micro": (64, 4, 2, 32, 4, 10), "tiny": (192, 3, 12, 64, 8, 10)}
    shas = {}
    for name, (D, H, L, img, B, nc) in specs.items():
        m, _ = ref_model(D, H, L, img, B, nc)
        shas[name] = {k: sha(v) for k, v in m.state_dict().items()}
        shas[name + "_keys"] = list(m.state_dict().keys())
    with open(os.path.join(HERE, "init_sha256.json"), "w") as f:
        json.dump(shas, f, indent=0)

    D, H, L, img, B, nc = specs["micro"]
    m, _ = ref_model(D, H, L, img, B, nc)
    x, y = batch(B, 3, img, nc)
    logits, loss, grads = run_eval_grads(m, x, y)
    np.savez_compressed(os.path.join(HERE, "micro.npz"), x=x.numpy(), y=y.numpy(), logits=logits.numpy(),
                        loss=loss.numpy(), **{"grad/" + k: v.numpy() for k, v in grads.items()})

    # ---------------- G4: tiny (C1) ----------------
    D, H, L, img, B, nc = specs["tiny"]
    m, _ = ref_model(D, H, L, img, B, nc)
    x, y = batch(B, 3, img, nc)
    logits, loss, grads = run_eval_grads(m, x, y)
    gnorm = {k: float(v.double().norm()) for k, v in grads.items()}
    # 3 AdamW steps (train.py:66,94-96) in eval mode on the same batch
    m, _ = ref_model(D, H, L, img, B, nc)
    m.eval()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    trace = []
    for _ in range(3):
        lg = m(x)
        ls = torch.nn.functional.cross_entropy(lg, y)
        opt.zero_grad(set_to_none=True)
        ls.backward()
        opt.step()
        trace.append(float(ls.item()))
    post = {k: float(v.double().norm()) for k, v in m.state_dict().items()}
    # the same 3 steps in fp64: the spread between the fp32 and fp64 traces is the reference's own sensitivity
    # (AdamW's first steps are ~lr*sign(g), so ~1e-7 gradient noise flips tiny components)
    m, _ = ref_model(D, H, L, img, B, nc)
    m = m.double().eval()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    trace64 = []
    for _ in range(3):
        ls = torch.nn.functional.cross_entropy(m(x.double()), y)
        opt.zero_grad(set_to_none=True)
        ls.backward()
        opt.step()
        trace64.append(float(ls.item()))
    m64, _ = ref_model(D, H, L, img, B, nc)
    m64 = m64.double().eval()
    logits64 = m64(x.double())
    torch.nn.functional.cross_entropy(logits64, y).backward()
    grads64 = {k: p.grad.detach().clone() for k, p in m64.named_parameters()}
    logits64 = logits64.detach()
    np.savez_compressed(os.path.join(HERE, "tiny.npz"), logits=logits.numpy(), logits64=logits64.numpy(),
                        loss=loss.numpy(), trace=np.array(trace), trace64=np.array(trace64),
                        gnorm_keys=np.array(list(gnorm.keys())), gnorm=np.array(list(gnorm.values())),
                        post_keys=np.array(list(post.keys())), post_norm=np.array(list(post.values())),
                        **{"gslice/" + k: v.reshape(-1)[::97].numpy() for k, v in grads.items()},
                        **{"gslice64/" + k: v.reshape(-1)[::97].numpy() for k, v in grads64.items()})

    # ---------------- G3: per-op KATs ----------------
    torch.manual_seed(7)
    ops = {}
    # Head (transformer.py:9-31): hd=16, D=64, B=2, T=5
    head = rtransformer.Head(16, 64, 5)
    xh = torch.randn(2, 5, 64, requires_grad=True)
    oh, wh = head(xh)
    go = torch.randn_like(oh)
    oh.backward(go)
    ops.update({"head/x": xh.detach().numpy(), "head/wq": head.query.weight.detach().numpy(),
                "head/wk": head.key.weight.detach().numpy(), "head/wv": head.value.weight.detach().numpy(),
                "head/out": oh.detach().numpy(), "head/wei": wh.detach().numpy(), "head/gout": go.numpy(),
                "head/dx": xh.grad.numpy()})
    # LayerNorm fwd/bwd (eps 1e-5)
    ln = torch.nn.LayerNorm(48)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    xl = (torch.randn(6, 48) * 3 + 1).requires_grad_(True)
    yl = ln(xl)
    gl = torch.randn_like(yl)
    yl.backward(gl)
    ops.update({"ln/x": xl.detach().numpy(), "ln/w": ln.weight.detach().numpy(), "ln/b": ln.bias.detach().numpy(),
                "ln/y": yl.detach().numpy(), "ln/gy": gl.numpy(), "ln/dx": xl.grad.numpy(),
                "ln/dw": ln.weight.grad.numpy(), "ln/db": ln.bias.grad.numpy()})
    # FeedForward in eval mode (ReLU)
    ff = rtransformer.FeedForward(32).eval()
    xf = torch.randn(3, 7, 32)
    ops.update({"ffn/x": xf.numpy(), "ffn/w1": ff.mlp[0].weight.detach().numpy(),
                "ffn/b1": ff.mlp[0].bias.detach().numpy(), "ffn/w2": ff.mlp[2].weight.detach().numpy(),
                "ffn/b2": ff.mlp[2].bias.detach().numpy(), "ffn/y": ff(xf).detach().numpy()})
    # CrossEntropy
    lg = torch.randn(5, 11)
    lb = torch.tensor([0, 3, 10, 7, 3])
    ops.update({"ce/logits": lg.numpy(), "ce/labels": lb.numpy(),
                "ce/loss": torch.nn.functional.cross_entropy(lg, lb).numpy()})
    # Dropout statistics of the reference (train mode): rate and scale
    mha = rtransformer.MultiHeadAttention(2, 8, 16, 5).train()
    d = mha.dropout(torch.ones(200000))
    ops.update({"dropout/zero_frac": np.array(float((d == 0).float().mean())),
                "dropout/nonzero_value": np.array(float(d[d != 0][0]))})
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **ops)

    # ---------------- G2: ViT-B width block ----------------
    res = {}
    for dt in (torch.float32, torch.float64):
        torch.manual_seed(11)
        blk = rtransformer.Block(768, 12, 197).eval().to(dt)
        g = torch.Generator().manual_seed(12)
        xb = torch.randn(2, 197, 768, generator=g, dtype=torch.float64).to(dt).requires_grad_(True)
        yb = blk(xb)
        gy = torch.randn(2, 197, 768, generator=torch.Generator().manual_seed(13), dtype=torch.float64).to(dt)
        yb.backward(gy)
        tag = "f32" if dt == torch.float32 else "f64"
        res[f"{tag}/y_slice"] = yb.detach().double().reshape(-1)[::101].numpy()
        res[f"{tag}/dx_slice"] = xb.grad.double().reshape(-1)[::101].numpy()
        res[f"{tag}/y_norm"] = np.array(float(yb.detach().double().norm()))
        res[f"{tag}/dx_norm"] = np.array(float(xb.grad.double().norm()))
        if dt == torch.float32:
            res["param_sha"] = np.array([sha(v) for v in blk.state_dict().values()])
    np.savez_compressed(os.path.join(HERE, "block_base.npz"), **res)

    print("goldens written to", HERE)


if __name__ == "__main__":
    main()
