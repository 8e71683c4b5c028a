"""Capture eval / mIoU golden vectors from the REFERENCE (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_eval_golden.py

Imports /root/reference/compute_iou.py (read-only; only its function definitions run) and
records, for deterministic synthetic label-id maps and predictions, the reference's
``label_mapping`` output, ``fast_hist`` confusion matrix and ``per_class_iu`` into
tests/golden/eval_goldens.npz.  The Cityscapes ``label2train`` list (dataset/cityscapes_list/
info.json) is absent from the reference tree; it is rebuilt from the id -> trainId map of
dataset/gta5_dataset.py:27-29 (other ids -> 255).  Only inputs/outputs are stored.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
OUT = os.path.join(HERE, "eval_goldens.npz")

# Cityscapes label2train: every id 0..33, the 19 train classes of dataset/gta5_dataset.py:27-29,
# every other id -> 255 (as in the Cityscapes devkit's info.json that compute_iou reads)
_TRAIN = {7: 0, 8: 1, 11: 2, 12: 3, 13: 4, 17: 5, 19: 6, 20: 7, 21: 8, 22: 9, 23: 10, 24: 11, 25: 12,
          26: 13, 27: 14, 28: 15, 31: 16, 32: 17, 33: 18}
MAPPING = np.array([[i, _TRAIN.get(i, 255)] for i in range(34)], dtype=np.int64)


def main():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    import compute_iou as ref  # noqa: E402

    rng = np.random.Generator(np.random.PCG64(77))
    out = {"mapping": MAPPING}
    for i, (h, w) in enumerate(((37, 53), (64, 128), (257, 129))):
        ids = rng.integers(0, 34, (h, w)).astype(np.uint8)
        ids[rng.uniform(0, 1, (h, w)) < 0.05] = 255  # unlabeled / void ids stay out of range
        pred = rng.integers(0, 19, (h, w)).astype(np.uint8)
        # make the prediction correlate with the ground truth so the IoUs are not all ~0
        mapped = ref.label_mapping(ids, MAPPING)
        agree = (rng.uniform(0, 1, (h, w)) < 0.6) & (mapped < 19)
        pred[agree] = mapped[agree].astype(np.uint8)
        hist = ref.fast_hist(mapped.flatten(), pred.flatten(), 19)
        out[f"ids{i}"], out[f"pred{i}"] = ids, pred
        out[f"mapped{i}"], out[f"hist{i}"] = mapped, hist.astype(np.int64)
        with np.errstate(divide="ignore", invalid="ignore"):
            out[f"iu{i}"] = ref.per_class_iu(hist.astype(np.float64))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, sorted(out))


if __name__ == "__main__":
    main()
