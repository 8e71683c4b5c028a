"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's evaluation / mIoU path.

Used as the checker of adaptsegnet_amd.evaluate (tests/, bench_eval's cpu_baseline); never
imported by the product path.  Pinned by tests/golden/eval_goldens.npz, captured from the
reference's own compute_iou functions (tests/golden/gen_eval_golden.py).

Restated reference code (file:line in /root/reference):
  prediction: interp(output2) -> argmax over classes -> uint8   evaluate_cityscapes.py:153-169
  fast_hist(a, b, n)                                            compute_iou.py:15-17
  per_class_iu(hist)                                            compute_iou.py:20-21
  label_mapping(input, mapping)                                 compute_iou.py:24-28
  mIoU = nanmean(per_class_iu(sum of hists))                    compute_iou.py:56-61
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def label_mapping(ids, mapping):
    """Every id listed in mapping[:, 0] becomes mapping[:, 1]; other values are kept."""
    out = np.array(ids, copy=True)
    for src, dst in mapping:
        out[ids == src] = dst
    return out.astype(np.int64)


def fast_hist(a, b, n):
    """Confusion counts hist[gt][pred] over pixels with 0 <= gt < n."""
    a = np.asarray(a).astype(np.int64).ravel()
    b = np.asarray(b).astype(np.int64).ravel()
    k = (a >= 0) & (a < n)
    return np.bincount(n * a[k] + b[k], minlength=n * n).reshape(n, n)


def per_class_iu(hist):
    hist = np.asarray(hist, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.diag(hist) / (hist.sum(1) + hist.sum(0) - np.diag(hist))


def miou(hist):
    return float(np.nanmean(per_class_iu(hist)))


def predict_argmax(logits, out_hw):
    """[N, C, h, w] logits -> uint8 [N, H, W]: bilinear (align_corners=True) to out_hw, then
    the first maximal class (numpy argmax semantics), computed in fp64."""
    up = F.interpolate(logits.double(), size=tuple(out_hw), mode="bilinear", align_corners=True)
    return up.argmax(dim=1).to(torch.uint8), up
