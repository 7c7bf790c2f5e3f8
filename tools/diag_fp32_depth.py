"""Where does the fp32 engine's full-depth ViT-B gradient error come from?  (round 5 diagnostic)
Per-tensor errors vs the fp64 oracle for the engine with and without the pruned last block, next to the fp32 and
sequential-chain oracles; then each block teacher-forced in fp32 (the fp64 oracle's block input and output gradient
fed to Engine.block_forward / block_backward) against the fp64 block.
    python tools/diag_fp32_depth.py [--batch 8] [--blocks 12]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-transformer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from oracle import vit_oracle as O  # noqa: E402
from VisionTransformer import config, vit  # noqa: E402
from VisionTransformer.optim import cross_entropy  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--blocks", type=int, default=12)
    args = ap.parse_args()
    ocfg = O.make_config("base", img=224, batch=args.batch, num_classes=1000, blocks=args.blocks)
    st = O.init_state(ocfg, seed=31)
    x, y = O.synthetic_batch(ocfg)
    xd, yd = x.to(DEV), y.to(DEV)
    sd = {k: v.to(DEV) for k, v in st.items()}
    _, _, g64 = O.loss_and_grads(sd, xd, yd, ocfg, dtype=torch.float64)
    _, _, g32 = O.loss_and_grads(sd, xd, yd, ocfg)
    res = {}
    for prune in (True, False):
        c = config.ViTConfig(3, 1000, ocfg.num_patches, 768, 16, 12, args.blocks, "cpu", args.batch)
        m = vit.VisionTransformer(c)
        m.load_state_dict(st)
        m = m.to(DEV).eval()
        m.hip_engine.prune_last = prune
        cross_entropy(m(xd), yd).backward()
        res[prune] = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    rows = []
    for k in g64:
        rows.append((rel(res[True][k], g64[k]), rel(res[False][k], g64[k]), rel(g32[k], g64[k]), k))
    rows.sort(key=lambda r: -r[0] / max(r[2], 1e-12))
    print("per-tensor error vs fp64: pruned, unpruned, oracle fp32 (worst 25 by pruned / oracle)")
    for r in rows[:25]:
        print(f"  {r[0]:.3e} {r[1]:.3e} {r[2]:.3e}  {r[3]}")
    # teacher-forced fp32 blocks
    e = O.embed_forward({k: v.double() for k, v in sd.items()}, xd.double(), ocfg).detach().requires_grad_(True)
    S64 = {k: v.double() for k, v in sd.items()}
    ins, outs = [], []
    for l in range(ocfg.num_blocks):
        ins.append(e)
        e, _ = O.block_forward(S64, l, e, ocfg)
        e.retain_grad()
        outs.append(e)
    torch.nn.functional.cross_entropy(O.head_forward(S64, e), yd).backward()
    c = config.ViTConfig(3, 1000, ocfg.num_patches, 768, 16, 12, args.blocks, "cpu", args.batch)
    m = vit.VisionTransformer(c)
    m.load_state_dict(st)
    m = m.to(DEV).eval()
    eng = m.hip_engine
    eng.ensure_ready(xd.device)
    req = {k: True for k in eng.owners}
    B, T, D = args.batch, ocfg.T, 768
    M = B * T
    print("teacher-forced fp32 blocks vs fp64 block: out, dx, worst weight gradient")
    for l in range(ocfg.num_blocks):
        xin = ins[l].detach().float().view(M, D).contiguous()
        dy = outs[l].grad.detach().float().view(M, D).contiguous()
        xo, saved = eng.block_forward(l, xin, B, False, 0, True)
        eng.G.zero_()
        dxi, _ = eng.block_backward(l, saved, dy, dy, False, 0.0, req, None, False, B)
        torch.cuda.synchronize()
        pre = f"transformer_encoder.blocks.{l}."
        p = {k: v.clone().requires_grad_(True) for k, v in S64.items() if k.startswith(pre)}
        xi = ins[l].detach().clone().requires_grad_(True)
        yo, _ = O.block_forward(p, l, xi, ocfg)
        yo.backward(outs[l].grad.detach())
        gref = {"fc1_w": p[pre + "ffwd.mlp.0.weight"].grad, "fc2_w": p[pre + "ffwd.mlp.2.weight"].grad,
                "ln2_w": p[pre + "ln2.weight"].grad, "ln1_w": p[pre + "ln1.weight"].grad,
                "proj_w": p[pre + "multi_head.proj.weight"].grad}
        errs = {n: rel(eng.gw[f"{l}.{n}"], gref[n]) for n in gref}
        print(f"  block {l}: out {rel(xo.view(B, T, D), yo):.2e} dx {rel(dxi.view(B, T, D), xi.grad):.2e} "
              + " ".join(f"{n} {v:.2e}" for n, v in errs.items()))


if __name__ == "__main__":
    main()
