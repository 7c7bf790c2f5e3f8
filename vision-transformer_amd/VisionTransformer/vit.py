"""PatchEmbedding and VisionTransformer — drop-in for src/VisionTransformer/vit.py.

Same constructors, attribute names (including the reference's `emdeddings` spelling), parameters, state_dict keys and
init draw order as the reference (vit.py:9-80).  `VisionTransformer.forward` runs the fused MI355X engine
(`_engine.Engine`): patch im2col + MFMA GEMM with bias/pos epilogue, L encoder blocks of fused kernels, and the
classifier MLP on token 0 (the first PATCH token, because the CLS token is appended last — vit.py:41,80).

Extra (additive) API:
  * `model.compute_dtype` — from ViTConfig (bf16 or fp32 arithmetic);
  * `model.store_attention_probs` — each block's `multi_head.attention_probs` [B, H, T, T] (transformer.py:48, which
    the reference fills on every forward).  None (default) = auto: filled whenever all blocks' probabilities
    together take at most `ATTENTION_PROBS_AUTO_BYTES` (256 MiB: C1 always, ViT-B/16 224² up to 12 images), left
    None above that (ViT-B/16 B=256 would write 477 MB per layer per step).  A forward that stores them runs the
    probability-writing attention kernel and no query-0 / two-chain shortcuts; set False for small-batch latency
    runs.  True / False force it on / off;
  * `model.enable_data_parallel(group=None, force=False)` — all-reduce (average) gradients over `torch.distributed`
    (RCCL) bucket-by-bucket while the backward is still running.  Use this instead of wrapping the model in
    `torch.nn.parallel.DistributedDataParallel` (which is detected and refused: the fused engine is one autograd
    node, so DDP's per-parameter reducer hooks would never fire);
  * `model.hip_engine` — the engine (flat gradient / shadow-weight buffers).  After writing the fp32 parameters
    out-of-band (through `p.data`, which autograd does not version), call `model.hip_engine.repack()`;
    `load_state_dict` and in-place writes on the parameters themselves are detected automatically.

Device semantics (the reference picks 'cuda' or 'cpu', train.py:26): a model on a ROCm device runs the fused HIP
engine and fails loudly when libvit_hip.so is missing; a model on the CPU runs the host path `_cpu.py` (plain torch
ops, standard autograd).  A CUDA input never falls back to the host path.

Gradient semantics kept from the reference module: `requires_grad=False` parameters get no gradient (`.grad` stays
None and their weight-gradient GEMMs are skipped), `x.requires_grad` yields the input gradient, and parameter hooks
(`register_hook`, `register_post_accumulate_grad_hook`) run once per backward, after the gradients are complete.
"""
import os

import torch
import torch.nn as nn

from . import _cpu
from . import _functional as Fh
from . import config as _config  # noqa: F401  (reference module imports config alongside transformer)
from . import transformer
from ._engine import Engine, ViTFunction

# store_attention_probs=None (auto) fills attention_probs when B * H * T^2 * 4 bytes * blocks fits in this budget
# (environment VIT_ATTENTION_PROBS_AUTO_BYTES overrides it, and reaches spawned worker processes too)
ATTENTION_PROBS_AUTO_BYTES = int(os.environ.get("VIT_ATTENTION_PROBS_AUTO_BYTES", 256 << 20))


class PatchEmbedding(nn.Module):
    def __init__(self, input_channels, embedding_size, patch_size, batch_size, num_patches, precision, device):
        super().__init__()
        # master weights are fp32 regardless of `precision` (which selects the compute dtype instead)
        self.sequence = nn.Sequential(
            nn.Conv2d(in_channels=input_channels, out_channels=embedding_size, kernel_size=patch_size,
                      stride=patch_size, device=device, dtype=torch.float32),
            nn.Flatten(2),
        )
        self.cls_tkn_embd = nn.Parameter(torch.randn(size=(batch_size, 1, embedding_size), device=device),
                                         requires_grad=True)
        self.pos_embd = nn.Parameter(torch.randn(size=(1, num_patches + 1, embedding_size), device=device),
                                     requires_grad=True)
        self.patch_size = patch_size
        self.compute_dtype = precision if precision in (torch.float32, torch.bfloat16) else torch.float32

    def forward(self, x):
        conv = self.sequence[0]
        return Fh.patch_embed(x, conv.weight, conv.bias, self.cls_tkn_embd, self.pos_embd, self.patch_size,
                              self.compute_dtype)


class VisionTransformer(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.vit_config = config
        self.compute_dtype = getattr(config, "compute_dtype", None) or (
            config.precision if config.precision in (torch.float32, torch.bfloat16) else torch.float32)
        self.emdeddings = PatchEmbedding(
            input_channels=config.input_channels,
            embedding_size=config.embedding_size,
            patch_size=config.patch_size,
            num_patches=config.num_patches,
            precision=self.compute_dtype,
            batch_size=config.batch_size,
            device=config.device,
        )
        self.transformer_encoder = transformer.TransformerEncoder(
            embedding_size=config.embedding_size,
            num_heads=config.num_heads,
            num_blocks=config.num_blocks,
            block_size=config.num_patches + 1,
        )
        self.mlp = nn.Sequential(
            nn.Linear(config.embedding_size, 4 * config.embedding_size),
            nn.GELU(),
            nn.LayerNorm(4 * config.embedding_size),
            nn.Linear(4 * config.embedding_size, config.num_classes),
        )
        self.store_attention_probs = None        # auto (module docstring); True / False force it
        self._engine = None
        self._anchor = None

    @property
    def hip_engine(self):
        if self._engine is None:
            self._engine = Engine(self)
        return self._engine

    def enable_data_parallel(self, group=None, force=False, grad_dtype=torch.float32, launch_mode="auto"):
        """Average gradients across the process group with RCCL, bucketed per block, overlapped with backward.
        `force` keeps the all-reduce path on even for a world of one rank (tests the collective on one GPU).
        `grad_dtype=torch.bfloat16` sends each bucket as bf16 (half the xGMI ring bytes): the fp32 gradients are
        rounded to bf16, averaged in bf16 and widened back; master weights and optimizer state stay fp32.
        `launch_mode` of the backward's GEMMs and fused attention backward beside the collectives: "shared" (one
        workgroup per item, VIT_FLAG_SHARED_CUS), "persistent" (one workgroup per CU) or "auto" = persistent: with
        CU-holding kernels beside the backward in place of RCCL's (tools/cu_hog_ab.py) the persistent grids stayed
        0.2-0.3 ms/step faster than the shared-CU launch, whose own cost is 0.4-0.7 ms/step (no N > 1
        measurement exists yet).  Results are bitwise the same in every mode."""
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("enable_data_parallel: torch.distributed is not initialised")
        if grad_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("enable_data_parallel: grad_dtype must be torch.float32 or torch.bfloat16")
        if launch_mode not in ("auto", "shared", "persistent"):
            raise ValueError("enable_data_parallel: launch_mode must be 'auto', 'shared' or 'persistent'")
        eng = self.hip_engine
        eng.ddp_group = group
        eng.comm_dtype = grad_dtype
        eng.ddp_enabled = bool(force) or dist.get_world_size(group) > 1
        # "shared": the backward's kernels launch one workgroup per item instead of a persistent one-per-CU grid
        # (VIT_FLAG_SHARED_CUS, vit_hip.h), so RCCL's all-reduce kernels beside them never wait for a whole grid
        eng.shared_cus = eng.ddp_enabled and launch_mode == "shared"
        # each replica draws its own dropout masks (the rank is folded into the forward's dropout seed)
        eng.dropout_rank = dist.get_rank(group) if eng.ddp_enabled else 0
        return self

    # the engine holds a weakref to its model and views of the parameters: never copy or pickle it (a deep copy or
    # an unpickled model builds its own engine on first use)
    def __getstate__(self):
        state = dict(super().__getstate__())
        state["_engine"] = None
        state["_anchor"] = None
        return state

    def __deepcopy__(self, memo):
        import copy
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__getstate__().items():
            object.__setattr__(new, k, copy.deepcopy(v, memo))
        return new

    def wants_attention_probs(self, batch):
        """Whether a forward over `batch` images fills every block's `multi_head.attention_probs`: the
        store_attention_probs setting, or with None (auto) whether they fit in ATTENTION_PROBS_AUTO_BYTES."""
        s = self.store_attention_probs
        if s is not None:
            return bool(s)
        c = self.vit_config
        T = c.num_patches + 1
        return batch * c.num_heads * T * T * 4 * c.num_blocks <= ATTENTION_PROBS_AUTO_BYTES

    def _check_not_ddp_wrapped(self):
        from torch.nn.parallel import DistributedDataParallel as DDP
        active = DDP._get_active_ddp_module()
        if active is not None and any(m is self for m in active.module.modules()):
            raise RuntimeError(
                "VisionTransformer must not be wrapped in torch.nn.parallel.DistributedDataParallel: the fused HIP "
                "engine is a single autograd node, so DDP's per-parameter reducer would never see the gradients. "
                "Call model.enable_data_parallel() instead (bucketed RCCL all-reduce overlapped with the backward).")

    def forward(self, x):
        if not x.is_cuda and all(not p.is_cuda for p in (self.mlp[3].weight, self.emdeddings.pos_embd)):
            return _cpu.vit_forward(self, x)              # host path: the model lives on the CPU (train.py:26)
        self._check_not_ddp_wrapped()
        eng = self.hip_engine
        want_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters()))
        if want_grad:
            if self._anchor is None or self._anchor.device != x.device:
                self._anchor = torch.zeros((), device=x.device, requires_grad=True)
            return ViTFunction.apply(x, self._anchor, eng, self.training, self.wants_attention_probs(x.shape[0]))
        logits, _ = eng.forward(x, self.training, save=False, want_probs=self.wants_attention_probs(x.shape[0]))
        return logits
