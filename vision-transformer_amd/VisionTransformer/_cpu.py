"""Host (CPU) path of the drop-in modules: what a model or module whose parameters live on the CPU runs.

The reference selects `device = 'cuda' if available else 'cpu'` (src/train.py:26) and trains wherever the model is
(train.py:80,89-96); BASELINE config 1 (ViT-Tiny/16 64^2 B8 fp32) is exactly that CPU run.  This module is the
package's own CPU implementation of the same arithmetic — NOT the oracle (oracle/ is test infrastructure and is never
imported here) and never a fallback for device tensors: it is reached only when both the input and the parameters
are CPU tensors (`vit.VisionTransformer.forward`, `_functional`).

It is written for the host's cores rather than mirrored from the reference's module structure:
  * the per-head key/query/value Linears of a block (transformer.py:12-18, one GEMM each per head) run as ONE GEMM
    against the concatenation of all heads' weights (rows: queries, keys, values), and the H per-head attention
    loops (transformer.py:44) as one batched scaled-dot-product attention with the reference's MULTIPLIED scale
    sqrt(hd) (transformer.py:24) — torch's fused CPU attention kernel;
  * `attention_probs` (transformer.py:48) is materialised as on the device path: per
    `model.wants_attention_probs(B)` (store_attention_probs, auto by size; [B, H, T, T] fp32 per block).
Standard autograd throughout, so requires_grad, hooks and torch DDP (gloo) behave as for any nn.Module.
"""
import torch
import torch.nn.functional as F

DROPOUT_P = 0.2          # transformer.py:35,53 (config.dropout is stored but unused by the reference)
LN_EPS = 1e-5


def _fused_qkv_weight(mh):
    """[3D, D]: query rows of every head, then keys, then values (the device engine's fused layout)."""
    heads = mh.heads
    return torch.cat([h.query.weight for h in heads] + [h.key.weight for h in heads] +
                     [h.value.weight for h in heads], dim=0)


def attention(a, w_qkv, H, want_probs=False):
    """softmax(q k^T * sqrt(hd)) v for all heads of a [B, T, D] input and fused weights [3*H*hd, D]; returns
    (o [B, T, H*hd], probs [B, H, T, T] or None)."""
    B, T, _ = a.shape
    hd = w_qkv.shape[0] // (3 * H)
    qkv = F.linear(a, w_qkv).view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)      # [3, B, H, T, hd]
    q, k, v = qkv[0], qkv[1], qkv[2]
    scale = float(hd) ** 0.5                                                  # multiplied (transformer.py:24)
    probs = None
    if want_probs:
        probs = torch.softmax((q @ k.transpose(-2, -1)) * scale, dim=-1)
        o = probs @ v
    else:
        o = F.scaled_dot_product_attention(q, k, v, scale=scale)
    return o.transpose(1, 2).reshape(B, T, H * hd), probs


def patch_embed(x, w, b, cls, pos, P):
    """Conv2d(k=s=P) -> flatten -> permute -> cat(CLS LAST) -> + pos (vit.py:21-29,39-42)."""
    e = F.conv2d(x.to(w.dtype), w, b, stride=P).flatten(2).transpose(1, 2)
    return torch.cat([e, cls.to(e.dtype)], dim=1) + pos


def block(blk, x, training, want_probs=False):
    """Pre-LN block (transformer.py:76-79): x + drop(proj(MHA(ln1 x))), then x + drop(FFN(ln2 x))."""
    mh = blk.multi_head
    a = F.layer_norm(x, (x.shape[-1],), blk.ln1.weight, blk.ln1.bias, LN_EPS)
    o, probs = attention(a, _fused_qkv_weight(mh), len(mh.heads), want_probs)
    mh.attention_probs = probs.detach() if probs is not None else None
    x = x + F.dropout(F.linear(o, mh.proj.weight, mh.proj.bias), DROPOUT_P, training)
    fc1, _, fc2, _ = blk.ffwd.mlp
    a = F.layer_norm(x, (x.shape[-1],), blk.ln2.weight, blk.ln2.bias, LN_EPS)
    h = torch.relu(F.linear(a, fc1.weight, fc1.bias))
    return x + F.dropout(F.linear(h, fc2.weight, fc2.bias), DROPOUT_P, training)


def vit_forward(model, x):
    """VisionTransformer.forward (vit.py:77-80) on the host: embeddings -> L blocks -> classifier on token 0."""
    emb = model.emdeddings
    conv = emb.sequence[0]
    if x.shape[0] != emb.cls_tkn_embd.shape[0]:
        raise RuntimeError(f"batch size {x.shape[0]} != config.batch_size {emb.cls_tkn_embd.shape[0]} "
                           "(the CLS token parameter is batch-shaped)")
    e = patch_embed(x, conv.weight, conv.bias, emb.cls_tkn_embd, emb.pos_embd, conv.kernel_size[0])
    for blk in model.transformer_encoder.blocks:
        e = block(blk, e, model.training, model.wants_attention_probs(x.shape[0]))
    fc0, _, ln, fc3 = model.mlp
    z = F.gelu(F.linear(e[:, 0, :], fc0.weight, fc0.bias))                  # token 0 = first PATCH (vit.py:80)
    z = F.layer_norm(z, (z.shape[-1],), ln.weight, ln.bias, LN_EPS)
    return F.linear(z, fc3.weight, fc3.bias)
