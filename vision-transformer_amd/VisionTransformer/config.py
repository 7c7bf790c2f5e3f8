"""ViTConfig — same constructor as the reference (src/VisionTransformer/config.py:7-29).

Differences, all optional / additive:
  * `compute_dtype` (new, keyword-only default None): the dtype the HIP kernels compute in.  None means "follow
    `precision`": float32 -> exact-fp32 path (fp32 MFMA), bfloat16 -> bf16 MFMA path with fp32 accumulation.
    In the reference `precision` only sets the Conv2d parameter dtype (vit.py:27); here master weights stay fp32
    (optimizer state is fp32) and `precision` selects the arithmetic of the whole network.
  * `dropout` is stored and, like the reference, not used: dropout is p = 0.2 at the two sites per block
    (transformer.py:35,53).
"""
import torch

PRESETS = {
    # name: (embedding_size, num_heads, num_blocks) — ViT-Ti/S/B/L with patch 16
    "tiny": (192, 3, 12),
    "small": (384, 6, 12),
    "base": (768, 12, 12),
    "large": (1024, 16, 24),
}


class ViTConfig:
    def __init__(self, input_channels, num_classes, num_patches, embedding_size, patch_size, num_heads, num_blocks,
                 device, batch_size, dropout=0.2, precision=torch.float32, *, compute_dtype=None):
        self.input_channels = input_channels
        self.num_classes = num_classes
        self.num_patches = num_patches
        self.embedding_size = embedding_size
        self.patch_size = patch_size
        self.num_heads = num_heads
        self.num_blocks = num_blocks
        self.dropout = dropout
        self.precision = precision
        self.device = device
        self.batch_size = batch_size
        if compute_dtype is None:
            compute_dtype = precision if precision in (torch.float32, torch.bfloat16) else torch.float32
        if compute_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"compute_dtype must be torch.float32 or torch.bfloat16, got {compute_dtype}")
        self.compute_dtype = compute_dtype

    @classmethod
    def preset(cls, name, img_size=224, patch_size=16, num_classes=1000, batch_size=256, device="cuda",
               input_channels=3, precision=torch.bfloat16, **kw):
        D, H, L = PRESETS[name]
        n = (img_size // patch_size) ** 2
        return cls(input_channels=input_channels, num_classes=num_classes, num_patches=n, embedding_size=D,
                   patch_size=patch_size, num_heads=H, num_blocks=L, device=device, batch_size=batch_size,
                   precision=precision, **kw)

    def __repr__(self):
        return (f"ViTConfig(C={self.input_channels}, classes={self.num_classes}, patches={self.num_patches}, "
                f"D={self.embedding_size}, P={self.patch_size}, heads={self.num_heads}, blocks={self.num_blocks}, "
                f"batch={self.batch_size}, compute={self.compute_dtype}, device={self.device})")
