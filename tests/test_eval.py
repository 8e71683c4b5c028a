"""Evaluation path: prediction maps and the mIoU confusion matrix.

* CPU: the oracle's label_mapping / fast_hist / per_class_iu reproduce the golden vectors
  captured from the reference's own compute_iou functions (tests/golden/gen_eval_golden.py),
  integer-exact.
* GPU (through the C ABI): the device confusion matrix equals the golden histograms exactly;
  the fused upsample+argmax equals the fp64 oracle's argmax at every pixel whose top-two
  interpolated scores differ by more than 1e-5 of the score range (fp32 vs fp64 rounding can
  only flip genuinely tied pixels), and such pixels are rare.
"""
import os

import numpy as np
import pytest
import torch

from oracle import reference_eval as E

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "eval_goldens.npz"))
DEV = "cuda"


def test_oracle_matches_reference_goldens():
    mapping = GOLD["mapping"]
    for i in range(3):
        mapped = E.label_mapping(GOLD[f"ids{i}"], mapping)
        assert np.array_equal(mapped, GOLD[f"mapped{i}"])
        hist = E.fast_hist(mapped, GOLD[f"pred{i}"], 19)
        assert np.array_equal(hist, GOLD[f"hist{i}"])
        iu = E.per_class_iu(hist)
        assert np.allclose(iu, GOLD[f"iu{i}"], equal_nan=True, rtol=0, atol=0)


def test_label_lut_is_label_mapping():
    from adaptsegnet_amd.evaluate import label_lut
    lut = label_lut(GOLD["mapping"], device="cpu").numpy()
    ids = GOLD["ids2"]
    assert np.array_equal(lut[ids], E.label_mapping(ids, GOLD["mapping"]))


def _ambiguous(up, top_gap):
    s = torch.sort(up, dim=1, descending=True).values
    rng = (up.amax() - up.amin()).item()
    return (s[:, 0] - s[:, 1]) <= top_gap * rng


@pytest.mark.gpu
def test_confusion_matrix_gpu():
    from adaptsegnet_amd.evaluate import ConfusionMatrix
    cm = ConfusionMatrix(19, GOLD["mapping"])
    total = np.zeros((19, 19), dtype=np.int64)
    for i in range(3):
        one = ConfusionMatrix(19, GOLD["mapping"])
        ids = torch.from_numpy(GOLD[f"ids{i}"]).to(DEV)
        pred = torch.from_numpy(GOLD[f"pred{i}"]).to(DEV)
        one.update(ids, pred)
        assert np.array_equal(one.numpy(), GOLD[f"hist{i}"])
        assert np.allclose(one.per_class_iu(), GOLD[f"iu{i}"], equal_nan=True, rtol=0, atol=0)
        cm.update(ids, pred)
        total += GOLD[f"hist{i}"]
    assert np.array_equal(cm.numpy(), total)
    assert cm.miou() == pytest.approx(E.miou(total), abs=0)
    # a large image: 1024x2048 per-block LDS bins + 64-bit merges stay exact
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 34, (1, 1024, 2048), generator=g, dtype=torch.uint8)
    pred = torch.randint(0, 19, (1, 1024, 2048), generator=g, dtype=torch.uint8)
    big = ConfusionMatrix(19, GOLD["mapping"])
    big.update(ids.to(DEV), pred.to(DEV))
    ref = E.fast_hist(E.label_mapping(ids.numpy(), GOLD["mapping"]), pred.numpy(), 19)
    assert np.array_equal(big.numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,out_hw", [((2, 19, 16, 32), (128, 256)), ((1, 19, 128, 256), (1024, 2048)),
                                          ((1, 5, 7, 9), (20, 33))])
def test_upsample_argmax_gpu(shape, out_hw):
    from adaptsegnet_amd.evaluate import upsample_argmax
    g = torch.Generator().manual_seed(11)
    logits = torch.randn(shape, generator=g, dtype=torch.float64) * 3
    ref, up = E.predict_argmax(logits, out_hw)
    got = upsample_argmax(logits.float().to(DEV).contiguous(memory_format=torch.channels_last), out_hw).cpu()
    diff = got != ref
    amb = _ambiguous(up, 1e-5)
    assert not (diff & ~amb).any(), int((diff & ~amb).sum())
    assert diff.sum().item() <= max(2, ref.numel() // 100000)


@pytest.mark.gpu
def test_predict_deeplab_multi_gpu():
    """evaluate_cityscapes.py:161-169 on the engine vs the oracle (eval-mode BN, fp64)."""
    from adaptsegnet_amd.evaluate import predict
    from adaptsegnet_amd.model import DeeplabMulti
    from oracle import reference_torch as R
    state = R.det_state(R.g_specs(), 1338)
    G = R.to_torch(state)
    x = torch.from_numpy(R.det_images((1, 3, 64, 96), 31))
    _, p2 = R.g_forward(G, x, (96, 64), train=False)   # upsampled to the input size, as `model(image)`
    m = DeeplabMulti(19)
    m.load_state_dict({k: torch.from_numpy(v.copy()) if v.dtype == np.int64 else torch.from_numpy(v.copy()).float()
                       for k, v in state.items()})
    m = m.to(DEV)
    out_hw = (128, 192)
    got = predict(m, x.float().to(DEV), out_hw).cpu()
    ref, up = E.predict_argmax(p2.detach(), out_hw)
    diff = got != ref
    amb = _ambiguous(up, 1e-3)  # fp32 network vs fp64: scores agree to ~1e-4 of their range
    assert not (diff & ~amb).any(), int((diff & ~amb).sum())
