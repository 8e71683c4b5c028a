"""CPU oracle of the GTA5 / Cityscapes input pipeline (test infrastructure only).

Restates /root/reference/dataset/gta5_dataset.py:47-71 (GTA5DataSet.__getitem__ minus file
I/O) in numpy:
  image.resize(crop_size, Image.BICUBIC)                         (:54)
  label.resize(crop_size, Image.NEAREST)                         (:55)
  id_to_trainid remap, 255 elsewhere, float32                    (:27-29, :61-63)
  RGB -> BGR, -= mean (IMG_MEAN of train_gta2cityscapes_multi.py:30), HWC -> CHW   (:65-68)
The resize arithmetic is Pillow's (a third-party dependency the reference calls; Pillow
12.2.0 is importable here): separable two-pass 8-bit resampling, horizontal pass first,
bicubic a = -0.5 with the support widened by the downscale factor, coefficients normalised
per output pixel and rounded to 22-bit fixed point, each pass rounded and clamped to uint8;
NEAREST = floor(box0 + (x + 0.5) * scale) accumulated in double.  The restatement is pinned
bit-exactly to Pillow itself by tests/test_data.py (and by the committed goldens in
tests/golden/data_goldens.npz for boxes without Pillow).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2
IMG_MEAN = np.array((104.00698793, 116.66876762, 122.67891434), dtype=np.float32)  # train:30
ID_TO_TRAINID = {7: 0, 8: 1, 11: 2, 12: 3, 13: 4, 17: 5, 19: 6, 20: 7, 21: 8, 22: 9, 23: 10, 24: 11,
                 25: 12, 26: 13, 27: 14, 28: 15, 31: 16, 32: 17, 33: 18}      # gta5_dataset.py:27-29


def bicubic(x: float) -> float:
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def resample_coeffs(in_size: int, out_size: int, support: float = 2.0):
    """Per output pixel: (xmin, n) and n fixed-point weights (int32), Pillow's precompute +
    8-bpc normalisation.  Returns bounds [out][2] int32 and kk [out][ksize] int32."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    sup = support * filterscale
    ksize = int(math.ceil(sup)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = int(center - sup + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + sup + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        w = [bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = sum(w)
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _pass(img: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """One 8-bpc resampling pass along `axis` (1 = horizontal, 0 = vertical) of an HxWxC uint8."""
    src = np.moveaxis(img, axis, 0).astype(np.int64)
    out = np.empty((bounds.shape[0],) + src.shape[1:], np.uint8)
    for o in range(bounds.shape[0]):
        x0, n = int(bounds[o, 0]), int(bounds[o, 1])
        acc = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for t in range(n):
            acc += src[x0 + t] * int(kk[o, t])
        acc = (acc.astype(np.int32)) >> PRECISION_BITS   # int32 wrap as Pillow's int ss
        out[o] = np.clip(acc, 0, 255).astype(np.uint8)
    return np.moveaxis(out, 0, axis)


def resize_bicubic(img: np.ndarray, size_wh) -> np.ndarray:
    """Pillow Image.resize(size, BICUBIC) of an HxWx3 uint8 RGB array."""
    h, w = img.shape[:2]
    ow, oh = size_wh
    out = img
    if ow != w:
        b, k = resample_coeffs(w, ow)
        out = _pass(out, b, k, 1)
    if oh != h:
        b, k = resample_coeffs(h, oh)
        out = _pass(out, b, k, 0)
    return out


def nearest_index(in_size: int, out_size: int) -> np.ndarray:
    """Source index of each output pixel for Image.resize(size, NEAREST): the affine
    transform's coordinate accumulated in double from (0.5 * scale), floored."""
    scale = in_size / out_size
    idx = np.empty(out_size, np.int32)
    v = 0.5 * scale
    for x in range(out_size):
        idx[x] = min(int(v), in_size - 1)
        v += scale
    return idx


def resize_nearest(lab: np.ndarray, size_wh) -> np.ndarray:
    ow, oh = size_wh
    yi = nearest_index(lab.shape[0], oh)
    xi = nearest_index(lab.shape[1], ow)
    return lab[yi][:, xi]


def label_lut(mapping=ID_TO_TRAINID, ignore=255) -> np.ndarray:
    lut = np.full(256, ignore, np.int32)
    for k, v in mapping.items():
        lut[k] = v
    return lut


def gta5_item(img_u8: np.ndarray, lab_u8: np.ndarray | None, crop_size, mean=IMG_MEAN):
    """GTA5DataSet.__getitem__ (:47-71) on decoded arrays: (CHW float32 BGR-mean image,
    float32 trainId label or None, size)."""
    image = resize_bicubic(img_u8, crop_size).astype(np.float32)
    label = None
    if lab_u8 is not None:
        label = label_lut()[resize_nearest(lab_u8, crop_size)].astype(np.float32)
    size = image.shape
    image = image[:, :, ::-1]
    image = image - np.asarray(mean, dtype=np.float32)    # float32 -= IMG_MEAN (float32, train:30)
    image = image.transpose((2, 0, 1))
    return image.copy(), label, np.array(size)
