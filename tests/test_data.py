"""Input pipeline (adaptsegnet_amd.data) — bit-exact parity.

CPU: the numpy restatement (oracle/reference_data.py) equals Pillow's own Image.resize
(BICUBIC / NEAREST) — the library the reference's GTA5DataSet.__getitem__ calls
(dataset/gta5_dataset.py:54-55) — and the committed goldens.  GPU: adaptseg_gta5_preprocess
equals the oracle (and Pillow) byte for byte on the image (float32, same fp32 subtraction
of IMG_MEAN) and exactly on the int64 labels, at GTA5's 1914x1052 -> 1280x720 and Cityscapes'
2048x1024 -> 1024x512, up-scaling, unchanged sizes and odd shapes.
"""
import os

import numpy as np
import pytest
import torch

from oracle import reference_data as D

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "data_goldens.npz")

SIZES = [((1052, 1914), (1280, 720)),   # GTA5 image -> input_size (train:48)
         ((1024, 2048), (1024, 512)),   # Cityscapes -> input_size_target
         ((37, 53), (80, 61)),          # up-scaling (filter support not widened)
         ((64, 96), (96, 64)),          # one axis unchanged (Pillow skips that pass)
         ((100, 130), (47, 33))]        # odd down-scaling


def _pil():
    try:
        from PIL import Image
        return Image
    except ImportError:  # pragma: no cover - the GPU box image has Pillow too
        return None


def _img(rng, h, w):
    """Natural-ish image: smooth ramps + noise + hard edges (exercises clamping)."""
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([(x * 255 // max(w - 1, 1)), (y * 255 // max(h - 1, 1)), ((x + y) % 256)], -1)
    noise = rng.integers(-40, 41, (h, w, 3))
    edges = ((x // 7 + y // 5) % 2) * 200
    return np.clip(base + noise + edges[..., None] - 100, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("hw,out", SIZES)
def test_oracle_resize_equals_pillow(hw, out):
    Image = _pil()
    if Image is None:
        pytest.skip("Pillow not importable")
    rng = np.random.default_rng(hash((hw, out)) % 2 ** 31)
    img = _img(rng, *hw)
    ref = np.asarray(Image.fromarray(img).resize(out, Image.BICUBIC))
    assert np.array_equal(D.resize_bicubic(img, out), ref)
    lab = rng.integers(0, 40, hw, dtype=np.uint8)
    lref = np.asarray(Image.fromarray(lab).resize(out, Image.NEAREST))
    assert np.array_equal(D.resize_nearest(lab, out), lref)


def test_oracle_matches_goldens():
    g = np.load(GOLDEN)
    for i in range(int(g["count"])):
        img, lab = g[f"img{i}"], g[f"lab{i}"]
        out = tuple(int(v) for v in g[f"size{i}"])
        image, label, _ = D.gta5_item(img, lab, out)
        assert np.array_equal(image, g[f"image{i}"])
        assert np.array_equal(label, g[f"label{i}"])


@pytest.mark.gpu
@pytest.mark.parametrize("hw,out", SIZES)
def test_gpu_preprocess_bit_exact(hw, out):
    from adaptsegnet_amd import data
    rng = np.random.default_rng(7 + hash((hw, out)) % 1000)
    n = 2
    imgs = np.stack([_img(rng, *hw) for _ in range(n)])
    labs = rng.integers(0, 40, (n,) + hw, dtype=np.uint8)
    dev = torch.device("cuda", 0)
    image, label = data.preprocess(torch.from_numpy(imgs).to(dev), torch.from_numpy(labs).to(dev), out)
    torch.cuda.synchronize()
    for b in range(n):
        ref_img, ref_lab, size = D.gta5_item(imgs[b], labs[b], out)
        got = image[b].cpu().numpy()
        assert got.dtype == np.float32 and got.shape == ref_img.shape
        assert np.array_equal(got.view(np.int32), ref_img.view(np.int32)), \
            f"{int((got != ref_img).sum())} pixels differ"
        assert np.array_equal(label[b].cpu().numpy(), ref_lab.astype(np.int64))
        assert tuple(size) == (out[1], out[0], 3)


@pytest.mark.gpu
def test_gpu_preprocess_image_only_and_errors():
    from adaptsegnet_amd import data
    dev = torch.device("cuda", 0)
    img = torch.from_numpy(_img(np.random.default_rng(1), 40, 60)[None]).to(dev)
    image, label = data.preprocess(img, None, (30, 20))
    assert label is None
    ref, _, _ = D.gta5_item(img[0].cpu().numpy(), None, (30, 20))
    assert np.array_equal(image[0].cpu().numpy(), ref)
    with pytest.raises(ValueError):
        data.preprocess(img.float(), None, (30, 20))
    with pytest.raises(ValueError):
        data.preprocess(img.cpu(), None, (30, 20))
