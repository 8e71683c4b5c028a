"""Checkpoint I/O (adaptsegnet_amd.checkpoint).

CPU: the pretrained remap of train_gta2cityscapes_multi.py:206-215 (first key component
dropped, 21-class layer5 skipped for 19 classes), the reference's snapshot names and stop
rule (:482-493, :705-719), and that snapshots load back with weights_only=True.
GPU: resume is exact — 2 steps, save_resume, a fresh trainer load_resume + 1 step equals 3
uninterrupted steps bit for bit (the kernels are deterministic: no float atomics).
"""
import os

import numpy as np
import pytest
import torch

from adaptsegnet_amd import checkpoint as C


def _g(num_classes=19):
    from adaptsegnet_amd.model import DeeplabMulti
    return DeeplabMulti(num_classes=num_classes)


def test_restore_from_remap_skips_layer5_for_19_classes():
    src = _g(21)
    with torch.no_grad():
        for i, p in enumerate(src.parameters()):
            p.fill_(0.001 * (i + 1))
    # the reference's RESTORE_FROM file (train:54) is a single-classifier DeepLab: trunk +
    # 21-class layer5, keys prefixed "Scale.", no layer6
    saved = {"Scale." + k: v.clone() for k, v in src.state_dict().items() if not k.startswith("layer6")}
    dst = _g(19)
    before = {k: v.clone() for k, v in dst.state_dict().items()}
    C.restore_from(dst, saved, num_classes=19)
    sd = dst.state_dict()
    for k, v in sd.items():
        if k.startswith("layer5"):
            assert torch.equal(v, before[k]), k          # 21-class classifier not copied
        elif k.startswith("layer6"):
            assert torch.equal(v, before[k]), k           # not in the pretrained file
        else:
            assert torch.equal(v, saved["Scale." + k]), k
    # 21 classes: layer5 is copied too
    dst21 = _g(21)
    C.restore_from(dst21, saved, num_classes=21)
    assert torch.equal(dst21.state_dict()["layer5.conv2d_list.0.weight"],
                       saved["Scale.layer5.conv2d_list.0.weight"])


class _Cfg:
    def __init__(self, level):
        self.level = level


class _Tr:
    def __init__(self, level):
        from adaptsegnet_amd.model import FCDiscriminator
        self.cfg = _Cfg(level)
        self.model = _g()
        self.D1 = FCDiscriminator(19) if level == "multi-level" else None
        self.D2 = FCDiscriminator(19)


@pytest.mark.parametrize("level", ["single-level", "multi-level"])
def test_snapshot_names_and_stop_rule(tmp_path, level):
    tr = _Tr(level)
    d = str(tmp_path)
    assert not C.snapshot_step(tr, d, 0, 5000, 150000)        # i_iter 0: nothing
    assert not C.snapshot_step(tr, d, 3, 5000, 150000)
    assert not os.listdir(d)
    assert not C.snapshot_step(tr, d, 5000, 5000, 150000)     # periodic snapshot
    sub = "single_level" if level == "single-level" else "multi_level"
    names = sorted(os.listdir(os.path.join(d, sub)))
    want = ["GTA5_5000.pth", "GTA5_5000_D2.pth"] + (["GTA5_5000_D1.pth"] if level == "multi-level" else [])
    assert names == sorted(want)
    assert C.snapshot_step(tr, d, 149999, 5000, 150000)       # final: GTA5_<num_steps_stop>
    assert os.path.exists(os.path.join(d, sub, "GTA5_150000.pth"))
    sd = torch.load(os.path.join(d, sub, "GTA5_5000.pth"), weights_only=True)
    ref = tr.model.state_dict()
    assert list(sd) == list(ref)
    for k in ref:
        assert sd[k].shape == ref[k].shape and torch.equal(sd[k], ref[k].cpu())


@pytest.mark.gpu
def test_resume_is_bit_exact(tmp_path):
    from test_model_gpu import build_g, build_d
    from oracle import reference_torch as R
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    dev = torch.device("cuda", 0)
    xs = torch.from_numpy(R.det_images((2, 3, 41, 57), 11)).float().to(dev)
    lab = torch.from_numpy(R.det_labels((2, 41, 57), 12)).to(dev)
    xt = torch.from_numpy(R.det_images((2, 3, 33, 49), 13)).float().to(dev)
    cfg = StepConfig(level="multi-level", gan="LS", input_size=(57, 41), input_size_target=(49, 33))

    def trainer():
        m, d1, d2 = build_g(), build_d(2001), build_d(2002)
        m.train()
        return AdaptSegTrainer(m, d1, d2, cfg)

    ref = trainer()
    for it in range(3):
        ref.step(it, [(xs, lab, xt)])
    a = trainer()
    for it in range(2):
        a.step(it, [(xs, lab, xt)])
    path = str(tmp_path / "resume.pth")
    C.save_resume(a, path, 1)
    b = trainer()
    start = C.load_resume(b, path)
    assert start == 2
    b.step(start, [(xs, lab, xt)])
    torch.cuda.synchronize()
    for mr, mb in ((ref.model, b.model), (ref.D1, b.D1), (ref.D2, b.D2)):
        sr, sb = mr.state_dict(), mb.state_dict()
        for k in sr:
            assert torch.equal(sr[k].cpu(), sb[k].cpu()), k
    assert np.isclose(ref.opt.param_groups[0]["lr"], b.opt.param_groups[0]["lr"])
