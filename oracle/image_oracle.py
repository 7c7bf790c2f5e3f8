"""ORACLE — CPU restatement of the reference's image transform.  TEST INFRASTRUCTURE ONLY (imported by tests/ only).

The reference's loader (src/train.py:151-155) is torchvision `Compose([Lambda(convert RGB), Resize((S, S)),
ToTensor()])` over PIL images (CIFAR10 at :157-159, BrainTumorDataset.py:35-39).  On a PIL image, torchvision's
Resize calls `PIL.Image.resize((S, S), BILINEAR)` (torchvision is absent here, so that is the documented call, not
code read from it); ToTensor is `uint8 / 255` as float32, CHW.  The resampling algorithm therefore lives in Pillow
(third-party, not vendored; Pillow 12.2.0 is importable in this image), whose published algorithm (libImaging
Resample.c, stable since Pillow 4.x) is restated here:

  per axis (in_size -> out_size): scale = in/out; filterscale = max(scale, 1); support = 1.0 * filterscale (triangle
  filter of radius 1); for output index i: center = (i + 0.5) * scale; lo = max(int(center - support + 0.5), 0);
  hi = min(int(center + support + 0.5), in_size); w_j = tri((j + lo - center + 0.5) / filterscale) for j < hi - lo,
  normalised by their (sequential double) sum, then fixed point k_j = int(0.5 + w_j * 2^22);
  horizontal pass first (each sample clip8((2^21 + sum k_j * px) >> 22), an 8-bit intermediate image), then the
  vertical pass the same way on it.

This restatement is pinned bit-exactly to Pillow itself (tests/test_image_pipeline.py); the GPU kernel
(vit_resize_to_tensor) is then checked against Pillow directly on the GPU box.
"""
import numpy as np

PRECISION_BITS = 22


def coeffs(in_size, out_size):
    """(bounds [out, 2] = (lo, count), fixed-point weights [out, ksize] int64) of Pillow's bilinear resampler."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(np.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int64)
    kk = np.zeros((out_size, ksize), dtype=np.int64)
    ss = 1.0 / filterscale
    for i in range(out_size):
        center = 0.0 + (i + 0.5) * scale
        lo = max(int(center - support + 0.5), 0)
        hi = min(int(center + support + 0.5), in_size) - lo
        w = []
        ww = 0.0
        for j in range(hi):
            t = abs(((j + lo) - center + 0.5) * ss)
            v = 1.0 - t if t < 1.0 else 0.0
            w.append(v)
            ww += v
        for j in range(hi):
            v = w[j] / ww if ww != 0.0 else w[j]
            kk[i, j] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[i] = (lo, hi)
    return bounds, kk


def _pass(img, axis, out_size):
    """One 8-bit resampling pass along `axis` (0 = rows / vertical, 1 = columns / horizontal) of [H, W, C] uint8."""
    in_size = img.shape[axis]
    if in_size == out_size:
        return img
    bounds, kk = coeffs(in_size, out_size)
    src = np.moveaxis(img.astype(np.int64), axis, 0)
    out = np.empty((out_size,) + src.shape[1:], dtype=np.uint8)
    for i in range(out_size):
        lo, n = bounds[i]
        acc = (1 << (PRECISION_BITS - 1)) + np.tensordot(kk[i, :n], src[lo:lo + n], axes=(0, 0))
        out[i] = np.clip(acc >> PRECISION_BITS, 0, 255)
    return np.moveaxis(out, 0, axis)


def to_rgb(img):
    """PIL convert('RGB') for raw L / LA / RGB / RGBA arrays ([H, W] or [H, W, C] uint8): replicate L, drop alpha."""
    if img.ndim == 2:
        img = img[:, :, None]
    c = img.shape[2]
    if c in (1, 2):
        return np.repeat(img[:, :, :1], 3, axis=2)
    return img[:, :, :3]


def resize_to_tensor(img, out_h, out_w):
    """RGB convert -> Pillow bilinear resize to (out_h, out_w) -> ToTensor: float32 [3, out_h, out_w]."""
    rgb = to_rgb(np.asarray(img, dtype=np.uint8))
    r = _pass(_pass(rgb, 1, out_w), 0, out_h)
    return (r.astype(np.float32) / np.float32(255.0)).transpose(2, 0, 1).copy()
