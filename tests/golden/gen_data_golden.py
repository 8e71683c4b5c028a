#!/usr/bin/env python3
"""Golden vectors for the input pipeline, generated with Pillow (the library the reference's
GTA5DataSet.__getitem__ calls, dataset/gta5_dataset.py:54-55) and the reference's own
post-processing steps (:57-68, IMG_MEAN of train_gta2cityscapes_multi.py:30), so boxes
without Pillow still pin oracle/reference_data.py.  The reference module itself cannot be
imported here (it imports torchvision and matplotlib); its arithmetic is restated below line
by line from :51-68.

    python tests/golden/gen_data_golden.py
"""
import os

import numpy as np
from PIL import Image

IMG_MEAN = np.array((104.00698793, 116.66876762, 122.67891434), dtype=np.float32)
ID_TO_TRAINID = {7: 0, 8: 1, 11: 2, 12: 3, 13: 4, 17: 5, 19: 6, 20: 7, 21: 8, 22: 9, 23: 10, 24: 11,
                 25: 12, 26: 13, 27: 14, 28: 15, 31: 16, 32: 17, 33: 18}


def item(img, lab, crop_size, mean=IMG_MEAN):
    image = Image.fromarray(img).resize(crop_size, Image.BICUBIC)
    label = Image.fromarray(lab).resize(crop_size, Image.NEAREST)
    image = np.asarray(image, np.float32)
    label = np.asarray(label, np.float32)
    label_copy = 255 * np.ones(label.shape, dtype=np.float32)
    for k, v in ID_TO_TRAINID.items():
        label_copy[label == k] = v
    image = image[:, :, ::-1]
    image -= mean
    image = image.transpose((2, 0, 1))
    return image.copy(), label_copy.copy()


def main():
    rng = np.random.default_rng(20261016)
    cases = [((53, 97), (64, 36)), ((30, 41), (57, 44)), ((48, 64), (48, 32))]
    out = {"count": np.array(len(cases))}
    for i, (hw, size) in enumerate(cases):
        img = rng.integers(0, 256, hw + (3,), dtype=np.uint8)
        lab = rng.integers(0, 40, hw, dtype=np.uint8)
        image, label = item(img, lab, size)
        out.update({f"img{i}": img, f"lab{i}": lab, f"size{i}": np.array(size), f"image{i}": image,
                    f"label{i}": label})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data_goldens.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


if __name__ == "__main__":
    main()
