"""Data path of the training loop — reference src/train.py:151-162 and src/BrainTumorDataset.py:10-39.

The reference decodes PIL images in 4 DataLoader workers and runs `Compose([convert('RGB'), Resize((S, S)),
ToTensor()])` on the host per image; its published run was loader-bound (~375 img/s).  Here the workers
only decode to raw uint8 HWC arrays and pack a batch into one byte buffer; the RGB conversion, the PIL-bilinear
resize and the /255 scaling run on the GPU in one kernel launch per batch (`vit_resize_to_tensor`, bit-exact with
Pillow), on a side stream one batch ahead of the training step.

  * `BrainTumorDataset(data_dir, train, test_size, transform, random_state)` — the reference's folder-per-class
    dataset with the same stratified split (BrainTumorDataset.py:10-32); `transform=None` returns the PIL image as
    the reference does, `transform=decode` returns the raw array for the GPU pipeline;
  * `CIFAR10Bin(root, train)` — CIFAR-10 from its binary distribution (cifar-10-batches-bin; no pickle, no network:
    the reference's `CIFAR10(download=True)` at train.py:157-159 cannot run offline);
  * `SyntheticRawImages` — deterministic uint8 images (optionally ragged sizes) for tests and benchmarks;
  * `collate_raw` / `raw_loader` — the packing collate and its DataLoader;
  * `GpuImageTransform(size)` — packed batch -> [B, 3, S, S] device tensor;
  * `DeviceBatches(loader, transform, device)` — iterates (images on device, labels on device), prefetching the next
    batch's copy + transform on a side stream;
  * `host_transform(size)` — the same transform on the host with Pillow (the CPU path, train.py --device cpu).
"""
import ctypes
import glob
import os

import numpy as np
import torch

from . import _lib

RAW_MODES = ("L", "LA", "RGB", "RGBA")


def decode(img):
    """PIL image -> uint8 [H, W] or [H, W, C] array the GPU pipeline converts to RGB itself (L / LA / RGB / RGBA);
    other modes (P, I;16, CMYK, ...) are converted to RGB here with Pillow, exactly as convert('RGB') would."""
    if img.mode not in RAW_MODES:
        img = img.convert("RGB")
    return np.asarray(img, dtype=np.uint8)


class BrainTumorDataset(torch.utils.data.Dataset):
    """Folder-per-class images with a stratified train/test split (reference BrainTumorDataset.py:10-39: classes are
    `os.listdir(data_dir)` in listing order, split by sklearn train_test_split(stratify=class, random_state))."""

    def __init__(self, data_dir, train=True, test_size=0.2, transform=None, random_state=42):
        import pandas as pd
        from sklearn.model_selection import train_test_split
        labels = os.listdir(data_dir)
        self.transform = transform
        self.data_dir = data_dir
        self.class_encoding = dict(enumerate(labels))
        rows = []
        for i, lab in enumerate(labels):
            rows += [(os.path.join(data_dir, lab, f), i) for f in os.listdir(os.path.join(data_dir, lab))]
        df = pd.DataFrame(rows, columns=["image", "class"])
        tr_x, ts_x, tr_y, ts_y = train_test_split(df[["image"]], df[["class"]], test_size=test_size,
                                                  stratify=df[["class"]], random_state=random_state)
        self.train = pd.concat([tr_x, tr_y], axis=1)
        self.test = pd.concat([ts_x, ts_y], axis=1)
        self.indexer = self.train if train else self.test

    def __len__(self):
        return self.indexer.shape[0]

    def __getitem__(self, idx):
        from PIL import Image
        path, label = self.indexer.iloc[idx]
        image = Image.open(path)
        if self.transform is not None:
            image = self.transform(image)
        return image, int(label)


class CIFAR10Bin(torch.utils.data.Dataset):
    """CIFAR-10 binary version: records of 1 label byte + 3072 bytes (R, G, B planes of 32x32).  Items are uint8
    [32, 32, 3] arrays (what PIL's Image.fromarray gives torchvision's CIFAR10) and int labels."""

    RECORD = 1 + 3 * 32 * 32

    def __init__(self, root, train=True):
        d = os.path.join(root, "cifar-10-batches-bin") if os.path.isdir(os.path.join(root, "cifar-10-batches-bin")) \
            else root
        files = sorted(glob.glob(os.path.join(d, "data_batch_*.bin"))) if train else [os.path.join(d, "test_batch.bin")]
        if not files or not all(os.path.exists(f) for f in files):
            raise FileNotFoundError(f"CIFAR-10 binary batches not found under {root} (no download: offline)")
        self.maps = [np.memmap(f, dtype=np.uint8, mode="r").reshape(-1, self.RECORD) for f in files]
        self.offsets = np.cumsum([0] + [m.shape[0] for m in self.maps])

    def __len__(self):
        return int(self.offsets[-1])

    def __getitem__(self, i):
        f = int(np.searchsorted(self.offsets, i, side="right")) - 1
        rec = self.maps[f][i - self.offsets[f]]
        return np.ascontiguousarray(rec[1:].reshape(3, 32, 32).transpose(1, 2, 0)), int(rec[0])


class SyntheticRawImages(torch.utils.data.Dataset):
    """Deterministic uint8 images: fixed `size` (H, W, C) or, with `ragged`, H and W drawn per item in
    [size/2, 2*size] (exercises the ragged-batch path)."""

    def __init__(self, n, size=(32, 32, 3), classes=10, seed=0, ragged=False):
        self.n, self.size, self.classes, self.seed, self.ragged = n, size, classes, seed, ragged

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        rng = np.random.default_rng(self.seed * 1000003 + i)
        h, w, c = self.size
        if self.ragged:
            h, w = int(rng.integers(h // 2, 2 * h + 1)), int(rng.integers(w // 2, 2 * w + 1))
        img = rng.integers(0, 256, size=(h, w, c), dtype=np.uint8)
        return img, int(rng.integers(0, self.classes))


def collate_raw(batch):
    """[(uint8 array [H, W] / [H, W, C], label)] -> (packed uint8 [total bytes], meta int64 [B, 4] = (offset, H, W,
    C), labels int64 [B]).  Runs in the DataLoader workers; the buffers are then pinned by the loader."""
    arrays = [np.ascontiguousarray(a, dtype=np.uint8) for a, _ in batch]
    meta = np.zeros((len(arrays), 4), dtype=np.int64)
    off = 0
    for i, a in enumerate(arrays):
        h, w = a.shape[:2]
        c = a.shape[2] if a.ndim == 3 else 1
        if c not in (1, 2, 3, 4):
            raise ValueError(f"image {i}: {c} channels (expected L, LA, RGB or RGBA)")
        meta[i] = (off, h, w, c)
        off += a.size
    packed = np.empty(off, dtype=np.uint8)
    for (o, _, _, _), a in zip(meta, arrays):
        packed[o:o + a.size] = a.reshape(-1)
    labels = torch.tensor([int(l) for _, l in batch], dtype=torch.int64)
    return torch.from_numpy(packed), torch.from_numpy(meta), labels


def raw_loader(dataset, batch_size, shuffle=True, num_workers=4, drop_last=True, pin_memory=True, sampler=None):
    """DataLoader yielding packed raw batches (train.py:161-162 uses 4 workers)."""
    return torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle and sampler is None,
                                       sampler=sampler, num_workers=num_workers, drop_last=drop_last,
                                       pin_memory=pin_memory, collate_fn=collate_raw,
                                       persistent_workers=num_workers > 0)


class GpuImageTransform:
    """convert('RGB') -> Resize((S, S)) (PIL bilinear) -> ToTensor on the GPU: packed batch -> [B, 3, S, S]."""

    def __init__(self, size, dtype=torch.float32):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.dtype = dtype
        self._ws = None

    def __call__(self, packed, meta, device=None, stream=None):
        meta_h = meta.cpu() if meta.is_cuda else meta
        B = meta_h.shape[0]
        sh, sw = self.size
        if B == 0:
            raise ValueError("empty batch")
        off, h, w, c = (meta_h[:, i] for i in range(4))
        if (h <= 0).any() or (w <= 0).any() or not ((c >= 1) & (c <= 4)).all():
            raise ValueError("invalid image metadata")
        if int((off + h * w * c).max()) > packed.numel() or (off < 0).any():
            raise ValueError("image metadata points outside the packed buffer")
        lib = _lib.load()
        ks = max(max(lib.vit_resize_ksize(int(a), sh) for a in h.unique()),
                 max(lib.vit_resize_ksize(int(a), sw) for a in w.unique()))
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        src = packed.to(dev, non_blocking=True)
        meta_d = meta_h.to(dev, non_blocking=True)
        need = lib.vit_resize_workspace_bytes(B, sh, sw, ks)
        if self._ws is None or self._ws.numel() < need or self._ws.device != dev:
            self._ws = torch.empty(max(need, 1 << 16), dtype=torch.uint8, device=dev)
        out = torch.empty(B, 3, sh, sw, dtype=self.dtype, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        code = _lib.F32 if self.dtype == torch.float32 else _lib.BF16
        _lib.check(lib.vit_resize_to_tensor(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(meta_d.data_ptr()), B,
                                            sh, sw, ks, ctypes.c_void_p(out.data_ptr()), code,
                                            ctypes.c_void_p(self._ws.data_ptr()), self._ws.numel(),
                                            ctypes.c_void_p(s.cuda_stream)), "vit_resize_to_tensor")
        if stream is not None:
            for t in (src, meta_d, self._ws):
                t.record_stream(stream)
        return out


class DeviceBatches:
    """Iterate a raw loader as (images [B, 3, S, S] on device, labels on device): the next batch's host->device copy
    and GPU transform are issued on a side stream while the caller's step runs on the current one."""

    def __init__(self, loader, transform, device):
        self.loader, self.transform, self.device = loader, transform, torch.device(device)

    def __len__(self):
        return len(self.loader)

    def _stage(self, batch, stream):
        packed, meta, labels = batch
        with torch.cuda.stream(stream):
            x = self.transform(packed, meta, self.device, stream=stream)
            y = labels.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        return x, y, ev

    def __iter__(self):
        side = torch.cuda.Stream(device=self.device)
        it = iter(self.loader)
        nxt = None
        try:
            nxt = self._stage(next(it), side)
        except StopIteration:
            return
        while nxt is not None:
            x, y, ev = nxt
            torch.cuda.current_stream(self.device).wait_event(ev)
            x.record_stream(torch.cuda.current_stream(self.device))
            y.record_stream(torch.cuda.current_stream(self.device))
            try:
                nxt = self._stage(next(it), side)
            except StopIteration:
                nxt = None
            yield x, y


class Transformed(torch.utils.data.Dataset):
    """(item, label) dataset with a per-item transform (the host path's Compose)."""

    def __init__(self, ds, tf):
        self.ds, self.tf = ds, tf

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, i):
        x, y = self.ds[i]
        return self.tf(x), y


def host_transform(size):
    """The reference transform on the host (Pillow): convert('RGB') -> resize((S, S), BILINEAR) -> /255 CHW."""
    sh, sw = (size, size) if isinstance(size, int) else size

    def tf(img):
        from PIL import Image
        if not isinstance(img, Image.Image):
            img = Image.fromarray(np.asarray(img, dtype=np.uint8))
        if img.mode != "RGB":
            img = img.convert("RGB")
        a = np.asarray(img.resize((sw, sh), Image.BILINEAR), dtype=np.uint8)
        return torch.from_numpy(a.astype(np.float32) / np.float32(255.0)).permute(2, 0, 1).contiguous()
    return tf
