"""Transformer encoder modules — drop-in for src/VisionTransformer/transformer.py.

Constructor signatures, sub-module names and parameter registration order are those of the reference, so
`state_dict()` keys, shapes and the random-init draw order are identical (verified bit-for-bit against the
reference in tests/test_dropin_cpu.py).  The arithmetic is not torch's: every forward here runs libvit_hip kernels
(module-level path, `_functional.py`) on ROCm tensors; on CPU tensors they run the host path (`_cpu.py`,
train.py --device cpu).  `VisionTransformer.forward` does not call these forwards at all — it runs
the fused whole-model engine (`_engine.py`) over the same parameters.

Reference semantics kept:
  * Head: separate key/query/value projections without bias; logits MULTIPLIED by sqrt(head_size); returns
    (out, wei) (transformer.py:20-31);
  * MultiHeadAttention: heads concatenated in order, proj(+bias), Dropout(0.2); `.attention_probs` holds the
    stacked per-head probabilities [B, H, T, T] after a forward (transformer.py:43-49);
  * FeedForward: Linear(D, 4D) -> ReLU -> Linear(4D, D) -> Dropout(0.2) (transformer.py:52-64);
  * Block: pre-LN, x + MHA(ln1(x)), x + FFN(ln2(x)), LayerNorm eps 1e-5 (transformer.py:66-79).
"""
import torch
import torch.nn as nn

from . import _functional as Fh
from ._ops import ACT_NONE, ACT_RELU


class Head(nn.Module):
    def __init__(self, head_size, n_embd, block_size):
        super().__init__()
        # registration order = reference draw order: key, query, value (transformer.py:12-18)
        self.key = nn.Linear(n_embd, head_size, bias=False)
        self.query = nn.Linear(n_embd, head_size, bias=False)
        self.value = nn.Linear(n_embd, head_size, bias=False)
        self.block_size = block_size

    def forward(self, x):
        return Fh.head_attention(x, self.query.weight, self.key.weight, self.value.weight)


_PROBS_WARNED = False


class MultiHeadAttention(nn.Module):
    def __init__(self, num_heads, head_size, n_embd, block_size, dropout=0.2):
        super().__init__()
        self.heads = nn.ModuleList([Head(head_size, n_embd, block_size) for _ in range(num_heads)])
        self.proj = nn.Linear(n_embd, n_embd)
        self._attention_probs = None
        self._probs_skipped = False     # set by the fused engine when it ran without storing probabilities
        self.dropout = nn.Dropout(dropout)

    @property
    def attention_probs(self):
        """[B, H, T, T] attention probabilities of the last forward (transformer.py:48).  The fused whole-model
        forward stores them per `model.wants_attention_probs(B)`: by default whenever they fit in
        vit.ATTENTION_PROBS_AUTO_BYTES, always with `model.store_attention_probs = True` (477 MB per layer at
        ViT-B/16 B=256); reading them after a fused forward that skipped them returns None and warns once."""
        global _PROBS_WARNED
        if self._attention_probs is None and self._probs_skipped and not _PROBS_WARNED:
            _PROBS_WARNED = True
            import warnings
            warnings.warn("MultiHeadAttention.attention_probs is None: the fused VisionTransformer forward skips the "
                          "attention probabilities above vit.ATTENTION_PROBS_AUTO_BYTES or with "
                          "`model.store_attention_probs = False`; set `model.store_attention_probs = True` to keep "
                          "them (the reference always stores them, transformer.py:48)", UserWarning, stacklevel=2)
        return self._attention_probs

    @attention_probs.setter
    def attention_probs(self, value):
        self._attention_probs = value
        self._probs_skipped = False

    def forward(self, x):
        pairs = [head(x) for head in self.heads]
        out = torch.cat([o for o, _ in pairs], dim=-1)
        out = Fh.linear(out, self.proj.weight, self.proj.bias, ACT_NONE)
        out = Fh.dropout(out, self.training, self.dropout.p)
        self.attention_probs = torch.stack([w for _, w in pairs], dim=1)
        return out


class FeedForward(nn.Module):
    def __init__(self, n_embd, dropout=0.2):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(n_embd, 4 * n_embd), nn.ReLU(), nn.Linear(4 * n_embd, n_embd),
                                 nn.Dropout(dropout))

    def forward(self, x):
        fc1, _, fc2, drop = self.mlp
        h = Fh.linear(x, fc1.weight, fc1.bias, ACT_RELU)          # ReLU fused in the GEMM epilogue
        y = Fh.linear(h, fc2.weight, fc2.bias, ACT_NONE)
        return Fh.dropout(y, self.training, drop.p)


class Block(nn.Module):
    def __init__(self, n_embd, n_head, block_size):
        super().__init__()
        head_size = n_embd // n_head
        self.multi_head = MultiHeadAttention(n_head, head_size, n_embd, block_size)
        self.ffwd = FeedForward(n_embd)
        self.ln1 = nn.LayerNorm(n_embd)
        self.ln2 = nn.LayerNorm(n_embd)

    def forward(self, x):
        x = x + self.multi_head(Fh.layer_norm(x, self.ln1.weight, self.ln1.bias))
        x = x + self.ffwd(Fh.layer_norm(x, self.ln2.weight, self.ln2.bias))
        return x


class TransformerEncoder(nn.Module):
    def __init__(self, embedding_size, num_heads, num_blocks, block_size):
        super().__init__()
        self.blocks = nn.Sequential(*[Block(embedding_size, num_heads, block_size) for _ in range(num_blocks)])

    def forward(self, x):
        return self.blocks(x)
