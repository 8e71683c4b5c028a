"""Evaluation on the HIP engine: prediction maps and the mIoU confusion matrix.

Restates the per-image body of /root/reference/evaluate_cityscapes.py:153-169 and the
metric of compute_iou.py:15-61:

* ``predict(model, images)``: eval-mode forward, ``interp`` to (1024, 2048) (bilinear,
  align_corners=True) and the class argmax, fused into ONE kernel that reads the 1/8-scale
  logits and writes one byte per output pixel (the reference materialises the 19x1024x2048
  fp32 upsampled map, copies it to the host and runs numpy argmax).
* ``ConfusionMatrix``: ``label_mapping`` (a 256-entry id -> trainId LUT) + ``fast_hist``
  accumulated on the device in int64; ``per_class_iu`` / ``miou`` on the 19x19 host copy.

Parity: tests/test_eval.py (golden vectors from the reference's compute_iou functions).
"""
from __future__ import annotations


import numpy as np
import torch

from . import kernels as K
from .ops import OPS

# Cityscapes id -> trainId (the devkit's label2train; 19 classes of dataset/gta5_dataset.py:27-29)
CITYSCAPES_TRAIN_IDS = {7: 0, 8: 1, 11: 2, 12: 3, 13: 4, 17: 5, 19: 6, 20: 7, 21: 8, 22: 9, 23: 10,
                        24: 11, 25: 12, 26: 13, 27: 14, 28: 15, 31: 16, 32: 17, 33: 18}


def label_lut(mapping=None, device="cuda") -> torch.Tensor:
    """int32[256] LUT of compute_iou.label_mapping: listed ids map, other ids keep their value.
    ``mapping``: iterable of (id, trainId) pairs; default = Cityscapes label2train (all 34 ids,
    void ids -> 255)."""
    if mapping is None:
        mapping = [(i, CITYSCAPES_TRAIN_IDS.get(i, 255)) for i in range(34)]
    lut = np.arange(256, dtype=np.int32)
    for src, dst in mapping:
        lut[int(src)] = int(dst)
    return torch.from_numpy(lut).to(device)


def upsample_argmax(logits: torch.Tensor, out_hw) -> torch.Tensor:
    """[N, C, h, w] fp32 logits (any layout) -> uint8 [N, H, W] class map."""
    if not logits.is_cuda or logits.dtype != torch.float32:
        raise RuntimeError("upsample_argmax: expected a float32 HIP tensor")
    x = K.nhwc_view(logits)
    n, h, w, c = x.shape
    oh, ow = int(out_hw[0]), int(out_hw[1])
    out = torch.empty((n, oh, ow), dtype=torch.uint8, device=logits.device)
    OPS.upsample_argmax(x, out)
    return out


@torch.no_grad()
def predict(model, images: torch.Tensor, out_hw=(1024, 2048)) -> torch.Tensor:
    """evaluate_cityscapes.py:158-169: DeeplabMulti -> output2, DeeplabVGG -> its single map."""
    model.eval()
    out = model(images)
    logits = out if getattr(model, "single_output", False) else out[1]
    return upsample_argmax(logits, out_hw)


class ConfusionMatrix:
    """Device-side ``hist += fast_hist(label_mapping(gt), pred, n)`` (compute_iou.py:54)."""

    def __init__(self, num_classes=19, mapping=None, device="cuda"):
        self.n = int(num_classes)
        self.hist = torch.zeros((self.n, self.n), dtype=torch.int64, device=device)
        self.lut = label_lut(mapping, device)

    def update(self, gt_ids: torch.Tensor, pred: torch.Tensor) -> None:
        """gt_ids: uint8 label-id map(s); pred: uint8 class map(s) of the same number of pixels.
        (compute_iou skips an image whose sizes differ; so does this: it raises.)"""
        if gt_ids.dtype != torch.uint8 or pred.dtype != torch.uint8:
            raise RuntimeError("ConfusionMatrix.update: uint8 label ids and predictions expected")
        if gt_ids.numel() != pred.numel():
            raise RuntimeError(f"ConfusionMatrix.update: {gt_ids.numel()} labels vs {pred.numel()} predictions")
        gt_ids, pred = gt_ids.contiguous(), pred.contiguous()
        OPS.confusion_hist(gt_ids, self.lut, pred, self.n, self.hist)

    def numpy(self) -> np.ndarray:
        return self.hist.cpu().numpy()

    def per_class_iu(self) -> np.ndarray:
        h = self.numpy().astype(np.float64)
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.diag(h) / (h.sum(1) + h.sum(0) - np.diag(h))

    def miou(self) -> float:
        return float(np.nanmean(self.per_class_iu()))
