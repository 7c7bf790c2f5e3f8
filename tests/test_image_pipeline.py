"""Loader path (reference src/train.py:151-162, src/BrainTumorDataset.py:10-39):
convert('RGB') -> Resize((S, S)) -> ToTensor, on the GPU (`vit_resize_to_tensor`) against Pillow itself.

Pillow is the third-party library the reference's transform runs (torchvision's Resize on PIL images calls
`Image.resize(size, BILINEAR)`; torchvision is absent here).  The CPU tests pin the restatement in
oracle/image_oracle.py bit-exactly to Pillow; the GPU tests compare the kernel with Pillow directly, bit-exact."""
import os

import numpy as np
import pytest
import torch

from oracle import image_oracle as IO

PIL = pytest.importorskip("PIL.Image")
Image = PIL

CASES = [  # (H, W, C, out_h, out_w): CIFAR 32 -> 224 / 256, downscale, identity axis, extreme ratios, tiny
    (32, 32, 3, 224, 224), (32, 32, 3, 256, 256), (300, 200, 3, 64, 64), (17, 45, 1, 224, 224),
    (97, 131, 4, 50, 333), (512, 512, 3, 224, 224), (64, 64, 3, 64, 64), (1000, 30, 2, 7, 99), (5, 5, 3, 256, 256),
    (224, 100, 3, 224, 224),
]
MODES = {1: "L", 2: "LA", 3: "RGB", 4: "RGBA"}


def _img(h, w, c, seed):
    a = np.random.default_rng(seed).integers(0, 256, size=(h, w, c), dtype=np.uint8)
    return a[:, :, 0] if c == 1 else a


def _pil_ref(a, oh, ow):
    """The reference transform: Lambda(convert RGB) -> Resize((oh, ow)) -> ToTensor (train.py:151-155)."""
    c = 1 if a.ndim == 2 else a.shape[2]
    im = Image.fromarray(a, mode=MODES[c])
    if im.mode != "RGB":
        im = im.convert("RGB")
    r = np.asarray(im.resize((ow, oh), Image.BILINEAR), dtype=np.uint8)
    return (r.astype(np.float32) / np.float32(255.0)).transpose(2, 0, 1)


@pytest.mark.parametrize("case", CASES)
def test_oracle_restatement_is_pillow_bit_exact(case):
    h, w, c, oh, ow = case
    a = _img(h, w, c, seed=h * 7 + w)
    np.testing.assert_array_equal(IO.resize_to_tensor(a, oh, ow), _pil_ref(a, oh, ow))


def test_collate_and_datasets(tmp_path):
    from VisionTransformer import data
    items = [(_img(5, 7, 3, 1), 3), (_img(4, 4, 1, 2), 1), (_img(2, 9, 4, 3), 0)]
    packed, meta, labels = data.collate_raw(items)
    assert meta.tolist() == [[0, 5, 7, 3], [105, 4, 4, 1], [121, 2, 9, 4]] and labels.tolist() == [3, 1, 0]
    assert packed.numel() == 121 + 72 and torch.equal(packed[105:121], torch.from_numpy(items[1][0].reshape(-1)))
    # CIFAR-10 binary layout: label byte + R, G, B planes
    rec = np.random.default_rng(0).integers(0, 256, size=(4, 3073), dtype=np.uint8)
    rec[:, 0] = [7, 1, 9, 0]
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rec[:2].tofile(d / "data_batch_1.bin")
    rec[2:].tofile(d / "data_batch_2.bin")
    rec[:1].tofile(d / "test_batch.bin")
    ds = data.CIFAR10Bin(str(tmp_path), train=True)
    assert len(ds) == 4 and len(data.CIFAR10Bin(str(tmp_path), train=False)) == 1
    img, lab = ds[2]
    assert lab == 9 and img.shape == (32, 32, 3)
    np.testing.assert_array_equal(img[:, :, 1], rec[2, 1 + 1024:1 + 2048].reshape(32, 32))
    # folder-per-class dataset, stratified split (BrainTumorDataset.py:10-32)
    root = tmp_path / "tumors"
    for cls, n in (("glioma", 10), ("none", 5)):
        (root / cls).mkdir(parents=True)
        for i in range(n):
            Image.fromarray(_img(20 + i, 30, 1, i)).save(root / cls / f"{i}.png")
    tr = data.BrainTumorDataset(str(root), train=True, test_size=0.2, transform=data.decode)
    te = data.BrainTumorDataset(str(root), train=False, test_size=0.2)
    assert len(tr) == 12 and len(te) == 3
    counts = {tr.class_encoding[c]: n for c, n in tr.indexer["class"].value_counts().items()}
    assert counts == {"glioma": 8, "none": 4}                 # stratified 80/20 per class
    x, y = tr[0]
    assert isinstance(x, np.ndarray) and x.ndim == 2 and y in (0, 1)
    assert te[0][0].mode == "L"                              # transform=None returns the PIL image, as the reference
    tf = data.host_transform(64)
    np.testing.assert_array_equal(tf(te[0][0]).numpy(), _pil_ref(np.asarray(te[0][0]), 64, 64))


@pytest.mark.gpu
@pytest.mark.parametrize("out", [(224, 224), (64, 48)])
def test_gpu_resize_matches_pillow_ragged_batch(out):
    """One launch over a ragged batch of every case's input size and mode: bit-exact with Pillow per image; the bf16
    output is the fp32 output rounded."""
    from VisionTransformer import data
    oh, ow = out
    items = [(_img(h, w, c, seed=i), i) for i, (h, w, c, _, _) in enumerate(CASES)]
    packed, meta, _ = data.collate_raw(items)
    x = data.GpuImageTransform((oh, ow))(packed, meta, device="cuda")
    xb = data.GpuImageTransform((oh, ow), dtype=torch.bfloat16)(packed, meta, device="cuda")
    torch.cuda.synchronize()
    for i, (a, _) in enumerate(items):
        np.testing.assert_array_equal(x[i].cpu().numpy(), _pil_ref(a, oh, ow), err_msg=str(CASES[i]))
    assert torch.equal(xb, x.bfloat16())


@pytest.mark.gpu
def test_gpu_pipeline_loader_end_to_end():
    """DataLoader (packing collate) -> DeviceBatches (side-stream H2D + transform, one batch ahead) == Pillow."""
    from VisionTransformer import data
    ds = data.SyntheticRawImages(12, size=(32, 32, 3), classes=10, seed=4, ragged=True)
    loader = data.raw_loader(ds, batch_size=4, shuffle=False, num_workers=0, pin_memory=True)
    got = []
    for x, y in data.DeviceBatches(loader, data.GpuImageTransform(64), "cuda"):
        got.append((x.cpu(), y.cpu()))
    assert len(got) == 3
    for b, (x, y) in enumerate(got):
        for j in range(4):
            a, lab = ds[4 * b + j]
            assert int(y[j]) == lab
            np.testing.assert_array_equal(x[j].numpy(), _pil_ref(a, 64, 64))
    with pytest.raises(ValueError):
        bad = torch.tensor([[0, 32, 32, 3]], dtype=torch.int64)
        data.GpuImageTransform(64)(torch.zeros(10, dtype=torch.uint8), bad, device="cuda")
