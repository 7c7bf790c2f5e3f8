"""ctypes binding of libvit_hip.so (include/vit_hip.h).

The library is built in-tree by `make -C vision-transformer_amd/csrc` (or `__graft_entry__.build()`).  It is loaded
AFTER `import torch`, so its DT_NEEDED libamdhip64.so.7 resolves to the HIP runtime torch already mapped.
There is deliberately no fallback: if the library is missing, every HIP-path call raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must be imported first: provides the HIP runtime the library binds to)

LIB_PATH = os.environ.get("VIT_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvit_hip.so")
ABI_VERSION = 14

F32, BF16, MASK4 = 0, 1, 2
FLAG_SHARED_CUS = 1          # VIT_FLAG_SHARED_CUS (vit_hip.h)
ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("a", ctypes.c_void_p), ("b", ctypes.c_void_p), ("c", ctypes.c_void_p),
        ("lda", ctypes.c_int64), ("ldb", ctypes.c_int64), ("ldc", ctypes.c_int64),
        ("m", ctypes.c_int64), ("n", ctypes.c_int64), ("k", ctypes.c_int64),
        ("a_kcontig", ctypes.c_int32), ("b_kcontig", ctypes.c_int32),
        ("in_dtype", ctypes.c_int32), ("out_dtype", ctypes.c_int32),
        ("alpha", ctypes.c_float), ("beta", ctypes.c_float),
        ("bias", ctypes.c_void_p),
        ("act", ctypes.c_int32), ("aux_dtype", ctypes.c_int32),
        ("aux", ctypes.c_void_p), ("ldaux", ctypes.c_int64),
        ("res", ctypes.c_void_p), ("ldres", ctypes.c_int64), ("res_rowmod", ctypes.c_int64),
        ("res_dtype", ctypes.c_int32),
        ("dropout_p", ctypes.c_float), ("dropout_seed", ctypes.c_uint32),
        ("split_k", ctypes.c_int32),
        ("out_group_rows", ctypes.c_int64), ("out_group_stride", ctypes.c_int64),
        ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_int64),
        ("colsum_part", ctypes.c_void_p),
        ("mask_out", ctypes.c_void_p),
        ("dropout_row_stride", ctypes.c_int64),
        ("flags", ctypes.c_int32),
        ("dropout_row0", ctypes.c_int64),
    ]


class ColsumJob(ctypes.Structure):
    _fields_ = [("part", ctypes.c_void_p), ("nparts", ctypes.c_int64), ("cols", ctypes.c_int64),
                ("nsets", ctypes.c_int32), ("out", ctypes.c_void_p * 3), ("beta", ctypes.c_float)]


class TensorChunk(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("shadow", ctypes.c_void_p), ("n", ctypes.c_int64)]


_P, _I64, _I32, _F, _U32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float, ctypes.c_uint32

# name: (restype, argtypes)
_SIGS = {
    "vit_abi_version": (ctypes.c_int, []),
    "vit_last_error": (ctypes.c_char_p, []),
    "vit_set_option": (ctypes.c_int, [ctypes.c_char_p, _I64]),
    "vit_get_option": (_I64, [ctypes.c_char_p]),
    "vit_gemm_workspace_bytes": (_I64, [ctypes.POINTER(GemmDesc)]),
    "vit_gemm": (ctypes.c_int, [ctypes.POINTER(GemmDesc), _P]),
    "vit_gemm_split_k_hint": (ctypes.c_int, [_I64, _I64, _I64, _I32]),
    "vit_im2col": (ctypes.c_int, [_P, _I32, _P, _I32, _I64, _I64, _I64, _I64, _I64, _P]),
    "vit_col2im": (ctypes.c_int, [_P, _I32, _P, _I32, _I64, _I64, _I64, _I64, _I64, _P]),
    "vit_embed_cls": (ctypes.c_int, [_P, _P, _P, _I32, _I64, _I64, _I64, _P]),
    "vit_layernorm_fwd": (ctypes.c_int, [_P, _I64, _P, _P, _P, _I64, _P, _P, _I64, _I64, _F, _I32, _P]),
    "vit_layernorm_bwd_parts": (_I64, [_I64, _I64]),
    "vit_layernorm_bwd": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _P, _P, _P, _F, _U32, _P, _P, _I32, _I64,
                                         _I64, _I32, _P]),
    "vit_attn_fwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _F, _I32, _I64, _P]),
    "vit_attn_bwd_uses_o32": (ctypes.c_int, [_I64, _I64, _I64, _I64, _I32]),
    "vit_attn_bwd_workspace_bytes": (_I64, [_I64, _I64, _I64, _I64, _I32]),
    "vit_attn_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _F, _I32, _P, _I32, _P]),
    "vit_attn_fwd_row0": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _F, _I32, _P]),
    "vit_attn_bwd_row0": (ctypes.c_int, [_P, _P, _I64, _P, _I64, _I64, _I64, _I64, _F, _I32, _P]),
    "vit_colsum_workspace_bytes": (_I64, [_I64, _I64]),
    "vit_colsum": (ctypes.c_int, [_P, _I64, _I32, _I64, _I64, _P, _F, _F, _P, _P]),
    "vit_colsum_finish": (ctypes.c_int, [_P, _I64, _I64, _I32, _P, _P, _P, _F, _P]),
    "vit_colsum_finish_batch": (ctypes.c_int, [ctypes.POINTER(ColsumJob), _I32, _P]),
    "vit_copy2d": (ctypes.c_int, [_P, _I64, _I32, _P, _I64, _I32, _I64, _I64, _I64, _I64, _F, _P]),
    "vit_dropout_bwd": (ctypes.c_int, [_P, _P, _I32, _I64, _F, _U32, _F, _P]),
    "vit_mask4_apply": (ctypes.c_int, [_P, _I64, _I32, _P, _I64, _I32, _P, _I64, _I64, _F, _P]),
    "vit_relu_bwd": (ctypes.c_int, [_P, _P, _P, _I32, _I64, _P]),
    "vit_gelu_fwd": (ctypes.c_int, [_P, _P, _I64, _P]),
    "vit_gelu_bwd": (ctypes.c_int, [_P, _P, _P, _I64, _P]),
    "vit_softmax_xent": (ctypes.c_int, [_P, _P, _I64, _I64, _P, _P, _P, _P]),
    "vit_resize_ksize": (ctypes.c_int, [_I64, _I64]),
    "vit_resize_workspace_bytes": (_I64, [_I64, _I64, _I64, _I64]),
    "vit_resize_to_tensor": (ctypes.c_int, [_P, _P, _I64, _I64, _I64, _I64, _P, _I32, _P, _I64, _P]),
    "vit_adamw": (ctypes.c_int, [_P, _I64, _F, _F, _F, _F, _F, _F, _F, _F, _I32, _P]),
    "vit_pack": (ctypes.c_int, [_P, _I64, _I32, _P]),
}

EXPORTED_SYMBOLS = tuple(_SIGS.keys())

_lib = None


class HipLibraryError(RuntimeError):
    pass


def load():
    """Load libvit_hip.so (once).  Raises HipLibraryError when it is missing or its ABI does not match."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HipLibraryError(f"{LIB_PATH} not found: build it with `make -C vision-transformer_amd/csrc` or "
                              "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.vit_abi_version()
    if v != ABI_VERSION:
        raise HipLibraryError(f"libvit_hip ABI version {v} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().vit_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


def call(name, *args):
    lib = load()
    check(getattr(lib, name)(*args), name)


def set_option(name, value):
    """vit_set_option (vit_hip.h): process-wide launch option of the library (kernel-variant choice for A/B runs and
    tests; defaults are the shipped configuration).  Returns the previous value."""
    lib = load()
    prev = lib.vit_get_option(name.encode())
    check(lib.vit_set_option(name.encode(), int(value)), f"vit_set_option({name!r})")
    return prev


def get_option(name):
    v = load().vit_get_option(name.encode())
    if v == -(1 << 63):
        raise KeyError(f"unknown libvit_hip option {name!r}")
    return v


class option:
    """Context manager: `with _lib.option("gemm_persist", 0): ...` sets an option and restores it on exit."""

    def __init__(self, name, value):
        self.name, self.value = name, value

    def __enter__(self):
        self.prev = set_option(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_option(self.name, self.prev)
        return False
