"""The plain-C batch-1 forward over the C-ABI (examples/vit_forward.c; SURVEY.md §8(f) row 4, the counterpart of the
reference's C prototype csrc/vit.c:443-484 / main :886-939) against the oracle.

The test writes the weights (the reference's state_dict order, oracle init) and one image as a VITW file, runs the C
program as a child process on the GPU and compares its logits with `oracle.forward` in eval mode:
  * fp32: logits within 1e-4 (relative norm) of the fp32 oracle — the same gate as the engine's fp32 parity tests;
  * bf16: within 2e-2 of the oracle that rounds to bf16 at this path's storage points (flash=True), as smoke() gates.
The binary is built by `make` in build() (vision-transformer_amd/csrc/Makefile), never inside a test.
"""
import os
import struct
import subprocess

import numpy as np
import pytest
import torch

from oracle import vit_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "vit_forward")
SRC = os.path.join(ROOT, "examples", "vit_forward.c")


def write_vitw(path, state, cfg, image):
    """VITW v1: int32 {magic, 1, C, img, P, D, H, L, nc}, the state_dict tensors in the reference order, the image."""
    keys = O.state_keys(cfg)
    with open(path, "wb") as f:
        f.write(struct.pack("<9i", 0x57544956, 1, cfg.input_channels, cfg.img_size, cfg.patch_size,
                            cfg.embedding_size, cfg.num_heads, cfg.num_blocks, cfg.num_classes))
        for k in keys:
            f.write(state[k].detach().float().contiguous().numpy().astype("<f4").tobytes())
        f.write(image.float().contiguous().numpy().astype("<f4").tobytes())


def vitw_floats(cfg):
    """Floats after the header, as examples/vit_forward.c counts them (its `total`)."""
    D, T, L, nc = cfg.embedding_size, cfg.num_patches + 1, cfg.num_blocks, cfg.num_classes
    F = 4 * D
    cpp = cfg.input_channels * cfg.patch_size ** 2
    blk = 3 * D * D + D * D + D + F * D + F + D * F + D + 4 * D
    return D + T * D + D * cpp + D + L * blk + F * D + F + 2 * F + nc * F + nc + cfg.input_channels * cfg.img_size ** 2


def _cfg(D, H, img, L, nc=10):
    c = O.make_config("micro", img=img, batch=1, blocks=L, num_classes=nc)
    c.embedding_size, c.num_heads = D, H
    return c


def test_vitw_layout_matches_the_c_reader(tmp_path):
    """The file the tests write is exactly the size the C program reads, for the shapes used below."""
    for D, H, img, L, nc in ((128, 2, 64, 2, 10), (768, 12, 224, 1, 1000)):
        cfg = _cfg(D, H, img, L, nc)
        st = O.init_state(cfg, seed=0)
        p = tmp_path / "w.bin"
        write_vitw(p, st, cfg, torch.zeros(cfg.input_channels, img, img))
        assert os.path.getsize(p) == 9 * 4 + 4 * vitw_floats(cfg)


def test_c_source_compiles_against_the_header(tmp_path):
    """The example is plain C11 over include/vit_hip.h and the HIP runtime API (no HIP device code)."""
    subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I/opt/rocm/include", "-I" + os.path.join(ROOT, "include"), SRC], check=True)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("shape", [(128, 2, 64, 2), (768, 12, 224, 1)], ids=["D128_L2", "base_width_L1"])
def test_c_forward_matches_oracle(tmp_path, dtype, shape):
    assert os.path.exists(EXE), "examples/vit_forward is built by build() (make in vision-transformer_amd/csrc)"
    D, H, img, L = shape
    cfg = _cfg(D, H, img, L, nc=10)
    st = O.init_state(cfg, seed=3)
    x = torch.randn(1, cfg.input_channels, img, img, generator=torch.Generator().manual_seed(11))
    wpath, lpath = tmp_path / "w.bin", tmp_path / "logits.bin"
    write_vitw(wpath, st, cfg, x[0])
    r = subprocess.run([EXE, str(wpath), str(lpath), dtype], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    got = torch.from_numpy(np.fromfile(lpath, dtype="<f4").copy())
    assert got.numel() == cfg.num_classes
    with torch.no_grad():
        if dtype == "f32":
            ref, tol = O.forward(st, x, cfg), 1e-4
        else:
            ref, tol = O.forward(st, x, cfg, bf16=True, flash=True), 2e-2
    err = float((got - ref[0]).norm() / ref[0].norm())
    assert err < tol, (dtype, shape, err, r.stdout)
