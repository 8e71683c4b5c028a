"""DeeplabVGG (config c4): module structure on CPU, fp32 HIP engine vs fp64 oracle on GPU.

The composition is pinned only by the restatement oracle/reference_torch.py:vgg_forward (the
reference module needs torchvision, absent here, and its pool-index line is Python 2 —
SURVEY.md §8c): parity of the composition is unpinned by the reference itself; every op in it
(3x3 dilated conv + bias, ReLU, 2x2 max-pool, ASPP) is pinned by the per-op goldens.

Stated tolerances: forward output rel-max <= 1e-4; weight / input gradients rel Frobenius
<= 1e-3 (fp32 accumulation over K up to 9*1024, plus rare ReLU-mask flips at |x| ~ 1e-7).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import reference_torch as R

DEV = "cuda"


def test_vgg_structure_cpu():
    from adaptsegnet_amd.model import DeeplabVGG
    m = DeeplabVGG(19)
    assert list(m.state_dict().keys()) == [k for k, _, _ in R.vgg_specs()]
    assert sum(p.numel() for p in m.parameters()) == 29573004
    prog = m.conv_program()
    assert [p for _, p in prog] == [c[4] for c in R.VGG_CONVS]
    assert [(c.dilation, c.padding) for c, _ in prog] == [(c[3], c[3]) for c in R.VGG_CONVS]
    assert len(list(m.optim_parameters(None))) == 38  # one group: self.parameters()
    assert [c.dilation for c in m.classifier_branches()] == [6, 12]


def test_vgg_oracle_shapes_cpu():
    P = R.to_torch(R.det_state(R.vgg_specs(), 7))
    x = torch.from_numpy(R.det_images((1, 3, 40, 56), 3))
    out = R.vgg_forward(P, x)
    assert out.shape == (1, 19, 5, 7)


def _sd(sd):
    return {k: torch.from_numpy(v.copy()).float() for k, v in sd.items()}


def _frob(a, b):
    a, b = a.detach().double().cpu().flatten(), b.detach().double().cpu().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(params=[(0, 0), (1, 0), (2, 0), (2, 512)], ids=["fp32", "wgrad-terms", "all-terms", "all-terms-c512"])
def vgg_terms(request, monkeypatch):
    """engine.VGG_TERMS: the VGG program on fp32 operands, with its weight gradients on the
    term-image kernel, or with every product reading term images — for every layer, or only
    where the tensors have >= 512 channels (engine.VGG_TERMS_MIN_C)."""
    from adaptsegnet_amd import engine
    monkeypatch.setattr(engine, "VGG_TERMS", request.param[0])
    monkeypatch.setattr(engine, "VGG_TERMS_MIN_C", request.param[1])
    return request.param


@pytest.mark.gpu
def test_vgg_forward_backward_gpu(vgg_terms):
    from adaptsegnet_amd.model import DeeplabVGG
    state = R.det_state(R.vgg_specs(), 4242)
    P = R.to_torch(state, trainable=lambda k: True)
    x = torch.from_numpy(R.det_images((2, 3, 72, 96), 5))
    xr = x.clone().requires_grad_(True)
    ref = R.vgg_forward(P, xr)
    g = torch.Generator().manual_seed(9)
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)

    m = DeeplabVGG(19)
    m.load_state_dict(_sd(state))
    m = m.to(DEV)
    xd = x.float().to(DEV).requires_grad_(True)
    out = m(xd)
    assert out.shape == ref.shape
    err = float((out.double().cpu() - ref.detach()).abs().max() / ref.detach().abs().max())
    assert err < 1e-4, err
    out.backward(gy.float().to(DEV).contiguous(memory_format=torch.channels_last))
    for name, p in m.named_parameters():
        if name.startswith(("classifier.conv2d_list.2", "classifier.conv2d_list.3")):
            assert p.grad is None, name  # the forward's early return never uses them
            continue
        f = _frob(p.grad, P[name].grad)
        assert f < 1e-3, (name, f)
    assert _frob(xd.grad, xr.grad) < 1e-3


@pytest.mark.gpu
def test_vgg_single_level_step_gpu(vgg_terms):
    """One c4-style trainer step: loss_seg2 = CE(interp(VGG(x))) matches the oracle, and the
    update touches every used parameter (SGD, one LR group) and no unused branch."""
    from adaptsegnet_amd.model import DeeplabVGG, FCDiscriminator
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    state = R.det_state(R.vgg_specs(), 4243)
    P = R.to_torch(state)
    x = torch.from_numpy(R.det_images((1, 3, 64, 80), 21))
    lab = torch.from_numpy(R.det_labels((1, 64, 80), 22))
    xt = torch.from_numpy(R.det_images((1, 3, 64, 80), 23))
    up = F.interpolate(R.vgg_forward(P, x), size=(64, 80), mode="bilinear", align_corners=True)
    ce_ref = float(R.cross_entropy2d(up, lab))

    m = DeeplabVGG(19)
    m.load_state_dict(_sd(state))
    m = m.to(DEV)
    d = FCDiscriminator(19).to(DEV)
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    cfg = StepConfig(level="single-level", input_size=(80, 64), input_size_target=(80, 64))
    tr = AdaptSegTrainer(m, None, d, cfg)
    losses = tr.step(0, [(x.float().to(DEV), lab.to(DEV), xt.float().to(DEV))]).values()
    assert abs(losses["loss_seg2"] - ce_ref) < 1e-4 * abs(ce_ref)
    for k, p in m.named_parameters():
        unused = k.startswith(("classifier.conv2d_list.2", "classifier.conv2d_list.3"))
        assert (p.grad is None) == unused, k
        if unused:
            assert torch.equal(before[k], p.detach()), k  # SGD skips grad-less params
    assert not torch.equal(before["features.0.weight"], m.features[0].weight.detach())
    assert np.isfinite(list(losses.values())).all()
