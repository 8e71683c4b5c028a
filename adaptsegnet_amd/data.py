"""Input pipeline: the reference's dataset classes with the per-image
arithmetic moved to the GPU.

Reference: dataset/gta5_dataset.py (GTA5DataSet) and the target loader the training script
builds (train_gta2cityscapes_multi.py:333-336, 520-523; ``dataset/cityscapes_dataset.py`` is
absent from the reference tree — its call site passes the same crop/mean/mirror arguments and
the loader is the image half of GTA5DataSet).

Split of the work:
  * ``__getitem__`` (DataLoader worker, CPU) only decodes the files, exactly as the reference
    opens them (``Image.open(img).convert('RGB')``, ``Image.open(label)``), and returns uint8
    arrays at the file's own size — no resize, remap or float conversion on the host;
  * ``preprocess`` (training process, GPU) runs the rest of __getitem__ (:54-68) on the whole
    batch in one library call (adaptseg_gta5_preprocess): Pillow-exact bicubic / nearest
    resize, id -> trainId LUT, RGB -> BGR, ``-= IMG_MEAN``, CHW — bit-identical to the
    reference's output (tests/test_data.py).
"""
from __future__ import annotations

import os.path as osp

import numpy as np
import torch

from .ops import OPS

IMG_MEAN = np.array((104.00698793, 116.66876762, 122.67891434), dtype=np.float32)  # train:30
ID_TO_TRAINID = {7: 0, 8: 1, 11: 2, 12: 3, 13: 4, 17: 5, 19: 6, 20: 7, 21: 8, 22: 9, 23: 10, 24: 11,
                 25: 12, 26: 13, 27: 14, 28: 15, 31: 16, 32: 17, 33: 18}      # gta5_dataset.py:27-29

_LUTS: dict = {}


def trainid_lut(device, mapping=None, ignore_label=255) -> torch.Tensor:
    """int32[256] id -> trainId table on ``device`` (255 for ids outside the mapping)."""
    mapping = ID_TO_TRAINID if mapping is None else mapping
    key = (str(device), tuple(sorted(mapping.items())), ignore_label)
    t = _LUTS.get(key)
    if t is None:
        lut = np.full(256, ignore_label, np.int32)
        for k, v in mapping.items():
            lut[k] = v
        t = _LUTS[key] = torch.from_numpy(lut).to(device)
    return t


def preprocess(images: torch.Tensor, labels: torch.Tensor | None = None, crop_size=(1280, 720),
               mean=IMG_MEAN, lut: torch.Tensor | None = None):
    """GTA5DataSet.__getitem__ :54-68 on a decoded batch, on the GPU.

    images: uint8 [n, H, W, 3] RGB (device); labels: uint8 [n, H, W] class ids or None.
    crop_size: (W, H) as the reference's ``crop_size``.  Returns (float32 [n, 3, h, w] BGR
    minus ``mean``, int64 [n, h, w] trainIds or None) — the reference's image / label after
    ``.long()`` (train:595)."""
    if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] != 3:
        raise ValueError("images must be uint8 [n, H, W, 3]")
    if not images.is_cuda:
        raise ValueError("preprocess runs on the GPU: move the decoded batch to the device first")
    images = images.contiguous()
    n, h, w, _ = images.shape
    ow, oh = crop_size
    out = torch.empty((n, 3, oh, ow), device=images.device, dtype=torch.float32)
    lab_out = None
    if labels is not None:
        if labels.dtype != torch.uint8 or tuple(labels.shape) != (n, h, w):
            raise ValueError("labels must be uint8 [n, H, W] matching images")
        labels = labels.contiguous()
        lab_out = torch.empty((n, oh, ow), device=images.device, dtype=torch.int64)
        if lut is None:
            lut = trainid_lut(images.device)
    m = np.asarray(mean, dtype=np.float32)
    OPS.gta5_preprocess(images, [float(m[0]), float(m[1]), float(m[2])], out, labels,
                        lut if labels is not None else None, lab_out)
    return out, lab_out


def _decode_rgb(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8)


def _decode_ids(path):
    from PIL import Image
    return np.asarray(Image.open(path), dtype=np.uint8)


class GTA5DataSet(torch.utils.data.Dataset):
    """Same constructor and file list as the reference (gta5_dataset.py:14-45).  Items are
    the decoded uint8 image / label at file size plus the name; ``collate`` stacks a batch of
    equally sized files and ``preprocess`` turns it into the reference's tensors on the GPU."""

    def __init__(self, root, list_path, max_iters=None, crop_size=(321, 321), mean=(128, 128, 128),
                 scale=True, mirror=True, ignore_label=255):
        self.root, self.list_path = root, list_path
        self.crop_size, self.scale, self.ignore_label = crop_size, scale, ignore_label
        self.mean, self.is_mirror = mean, mirror
        self.img_ids = [i_id.strip() for i_id in open(list_path)]
        if max_iters is not None:
            self.img_ids = self.img_ids * int(np.ceil(float(max_iters) / len(self.img_ids)))
        self.id_to_trainid = dict(ID_TO_TRAINID)
        self.files = [{"img": osp.join(root, "images/%s" % name), "label": osp.join(root, "labels/%s" % name),
                       "name": name} for name in self.img_ids]

    def __len__(self):
        return len(self.files)

    def __getitem__(self, index):
        f = self.files[index]
        return _decode_rgb(f["img"]), _decode_ids(f["label"]), f["name"]

    def preprocess(self, images, labels, device=None):
        """The device half of __getitem__ for a collated batch (numpy or tensors)."""
        dev = device or torch.device("cuda", torch.cuda.current_device())
        im = torch.as_tensor(images).to(dev, non_blocking=True)
        lb = torch.as_tensor(labels).to(dev, non_blocking=True)
        lut = trainid_lut(dev, self.id_to_trainid, self.ignore_label)
        return preprocess(im, lb, self.crop_size, self.mean, lut)


class cityscapesDataSet(torch.utils.data.Dataset):  # noqa: N801  (the reference's class name)
    """The target loader of train_gta2cityscapes_multi.py:333-336 / 520-523 (its module is
    absent from the reference tree): list of ``leftImg8bit/<set>/<name>`` images; items are the
    decoded uint8 image at file size, the device half resizes to ``crop_size`` (BICUBIC),
    flips to BGR and subtracts ``mean`` like GTA5DataSet's image path."""

    def __init__(self, root, list_path, max_iters=None, crop_size=(321, 321), mean=(128, 128, 128),
                 scale=True, mirror=True, ignore_label=255, set="val"):  # noqa: A002
        self.root, self.list_path, self.set = root, list_path, set
        self.crop_size, self.scale, self.ignore_label = crop_size, scale, ignore_label
        self.mean, self.is_mirror = mean, mirror
        self.img_ids = [i_id.strip() for i_id in open(list_path)]
        if max_iters is not None:
            self.img_ids = self.img_ids * int(np.ceil(float(max_iters) / len(self.img_ids)))
        self.files = [{"img": osp.join(root, "leftImg8bit/%s/%s" % (set, name)), "name": name}
                      for name in self.img_ids]

    def __len__(self):
        return len(self.files)

    def __getitem__(self, index):
        f = self.files[index]
        return _decode_rgb(f["img"]), f["name"]

    def preprocess(self, images, device=None):
        dev = device or torch.device("cuda", torch.cuda.current_device())
        im = torch.as_tensor(images).to(dev, non_blocking=True)
        return preprocess(im, None, self.crop_size, self.mean)[0]


def collate(batch):
    """Stack decoded items of one size: (uint8 [n,H,W,3], uint8 [n,H,W] or None, names)."""
    imgs = np.stack([b[0] for b in batch])
    if len(batch[0]) == 3:
        return imgs, np.stack([b[1] for b in batch]), [b[2] for b in batch]
    return imgs, None, [b[1] for b in batch]


__all__ = ["IMG_MEAN", "ID_TO_TRAINID", "preprocess", "trainid_lut", "GTA5DataSet", "cityscapesDataSet", "collate",
]
