"""MI355X-native drop-in for the reference `VisionTransformer` package (src/VisionTransformer/{config,transformer,
vit}.py): same classes, constructor signatures and state_dict keys; the arithmetic runs in hand-written gfx950 HIP
kernels (libvit_hip.so, C-ABI in include/vit_hip.h).  There is no CPU compute path."""
from . import config, transformer, vit  # noqa: F401
from .optim import CrossEntropyLoss, FusedAdamW, cross_entropy  # noqa: F401
