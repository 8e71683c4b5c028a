"""GPU parity of the fork's Warper path through the C ABI.

Stated tolerances (fp32 HIP vs fp64 CPU oracle / goldens captured from the reference):
  * up2_relu_cat fwd / bwd, BN with LeakyReLU and affine gradients: rel <= 2e-6 of max|ref|;
  * warp (grid_sample) output and input gradient: rel <= 1e-5; warp-field gradient: rel <= 1e-4
    (it is the derivative of a piecewise-bilinear map: fp32 rounding of the sample point moves
    the weights by ~1e-7 relative, amplified by size/2);
  * Warper forward: flow rel <= 2e-3, warp_list norms rel <= 1e-3 (14 train-mode BNs, the deepest
    over 8 values per channel); parameter gradients: cosine >= 0.999, rel Frobenius <= 2e-2;
  * source-only step with the warper: loss rel <= 1e-3, generator update cosine >= 0.99,
    accumulated warper gradients cosine >= 0.99.
The input gradient of the warp is a data-dependent scatter accumulated in 64-bit fixed point:
it must also be bitwise reproducible run to run.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import reference_torch as R
from oracle import reference_warper as RW

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(__file__), "golden", "warper_goldens.npz")
W_SEED, W_CONV_STD = 3001, 0.02
WARP_IN, WARP_FLOW = (2, 19, 16, 24), (2, 2, 16, 24)


def rel(a, b):
    a, b = torch.as_tensor(a).detach().double().cpu(), torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def frob(a, b):
    a, b = a.detach().double().cpu().flatten(), b.detach().double().cpu().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30)), float(F.cosine_similarity(a, b, dim=0))


def det_normal(shape, seed, scale=1.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(scale * rng.standard_normal(shape))


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def build_warper():
    from adaptsegnet_amd.model import Warper
    w = Warper()
    sd = R.det_state(RW.warper_specs(), W_SEED, conv_std=W_CONV_STD)
    w.load_state_dict({k: torch.from_numpy(v.copy()) if v.dtype == np.int64 else torch.from_numpy(v.copy()).float()
                       for k, v in sd.items()})
    return w.to(DEV)


@pytest.mark.parametrize("n,h,w,cs,cd", [(2, 5, 7, 8, 12), (1, 1, 1, 0, 512), (2, 4, 3, 0, 64), (1, 2, 2, 64, 64)])
def test_up2_relu_cat(n, h, w, cs, cd):
    from adaptsegnet_amd import kernels as K
    s = det_normal((n, cs, h, w), 31) if cs else None
    d = det_normal((n, cd, h, w), 32)
    g = det_normal((n, cs + cd, 2 * h, 2 * w), 33)
    s_ = s.clone().requires_grad_(True) if cs else None
    d_ = d.clone().requires_grad_(True)
    cat = d_ if not cs else torch.cat((s_, d_), 1)
    ref = F.interpolate(F.relu(cat), scale_factor=2, mode="bilinear", align_corners=False)
    (ref * g).sum().backward()
    sg = nhwc(s).float().to(DEV) if cs else None
    dg = nhwc(d).float().to(DEV)
    out = K.up2_relu_cat_fwd(sg, dg)
    assert rel(out.permute(0, 3, 1, 2), ref) < 2e-6
    ds, dd = K.up2_relu_cat_bwd(sg, dg, nhwc(g).float().to(DEV))
    assert rel(dd.permute(0, 3, 1, 2), d_.grad) < 2e-6
    if cs:
        assert rel(ds.permute(0, 3, 1, 2), s_.grad) < 2e-6


@pytest.mark.parametrize("act", [0, 1, 2])
def test_bn_act_and_affine_grads(act):
    from adaptsegnet_amd import kernels as K
    rows, c = 2 * 9 * 11, 64
    x = det_normal((rows, c), 41) * 3 + 1
    wt = 1 + 0.1 * det_normal((c,), 42)
    b = 0.1 * det_normal((c,), 43)
    dy = det_normal((rows, c), 44)
    xr, wr, br = x.clone().requires_grad_(True), wt.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = F.batch_norm(xr, None, None, wr, br, True, 0.1, 1e-5)
    y = [y, F.relu(y), F.leaky_relu(y, 0.2)][act]
    (y * dy).sum().backward()
    rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
    xg = x.float().to(DEV)
    yg, mean, invstd = K.bn_fwd_train(xg, wt.float().to(DEV), b.float().to(DEV), rm, rv, 0.1, 1e-5, relu=act)
    assert rel(yg, y) < 2e-6
    dwg, dbg = torch.full((c,), 0.5, device=DEV), torch.full((c,), -0.25, device=DEV)
    for y_src in (yg, None):   # mask from y, or recomputed from x
        dw, db = dwg.clone(), dbg.clone()
        dx = K.bn_bwd_affine(dy.float().to(DEV), y_src, xg, wt.float().to(DEV), b.float().to(DEV), mean, invstd,
                             act, dw, db)
        assert rel(dx, xr.grad) < 2e-5
        assert rel(dw - 0.5, wr.grad) < 2e-5 and rel(db + 0.25, br.grad) < 2e-5   # accumulated


@pytest.mark.parametrize("tag,scale", [("mod", 0.8), ("sat", 6.0)])
def test_grid_warp_matches_reference_goldens(tag, scale):
    from adaptsegnet_amd import kernels as K
    gold = np.load(GOLD)
    inp, fl, r = det_normal(WARP_IN, 23), det_normal(WARP_FLOW, 24, scale), det_normal(WARP_IN, 25)
    xg, fg, rg = nhwc(inp).float().to(DEV), nhwc(fl).float().to(DEV), nhwc(r).float().to(DEV)
    _, y = K.grid_warp_fwd(fg, None, xg)
    assert rel(y.permute(0, 3, 1, 2), gold[f"warp_{tag}/out"]) < 1e-5
    dflow, _, dx = K.grid_warp_bwd(fg, None, xg, None, rg)
    assert rel(dx.permute(0, 3, 1, 2), gold[f"warp_{tag}/d_input"]) < 1e-5
    assert rel(dflow.permute(0, 3, 1, 2), gold[f"warp_{tag}/d_flow"]) < 1e-4
    # bitwise reproducible scatter
    _, _, dx2 = K.grid_warp_bwd(fg, None, xg, None, rg, need_dflow=False)
    assert torch.equal(dx, dx2)
    # two heads sharing the field: the field gradient is the sum of both heads'
    y1, y2 = K.grid_warp_fwd(fg, xg, 2 * xg)
    assert torch.equal(y1, y) and rel(y2, 2 * y) < 1e-6
    dflow2, dx1, dx2b = K.grid_warp_bwd(fg, xg, 2 * xg, rg, rg)
    assert rel(dflow2.permute(0, 3, 1, 2), 3 * torch.from_numpy(gold[f"warp_{tag}/d_flow"])) < 1e-4
    assert torch.equal(dx1, dx) and torch.equal(dx2b, dx)


def test_resnetmulti_warp_autograd():
    """DeeplabMulti.warp (static) through autograd matches the oracle's warp in fp64."""
    from adaptsegnet_amd.model import ResNetMulti
    inp, fl = det_normal(WARP_IN, 23), det_normal(WARP_FLOW, 24, 0.8)
    a, f = inp.clone().requires_grad_(True), fl.clone().requires_grad_(True)
    ref = RW.warp(a, f)
    r = det_normal(ref.shape, 25)
    (ref * r).sum().backward()
    ag = nhwc(inp).float().to(DEV).permute(0, 3, 1, 2).requires_grad_(True)
    fg = nhwc(fl).float().to(DEV).permute(0, 3, 1, 2).requires_grad_(True)
    out = ResNetMulti.warp(ag, fg)
    (out * r.float().to(DEV)).sum().backward()
    assert rel(out, ref) < 1e-5 and rel(ag.grad, a.grad) < 1e-5 and rel(fg.grad, f.grad) < 1e-4


def test_warper_forward_backward():
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    P = R.to_torch(R.det_state(RW.warper_specs(), W_SEED, conv_std=W_CONV_STD), trainable=RW.warper_trainable)
    x = torch.from_numpy(R.det_images((2, 3, 256, 256), 21))
    flow_ref, wl_ref = RW.warper_forward(P, x, train=True)
    rw = det_normal(flow_ref.shape, 22)
    (flow_ref * rw).sum().backward()

    w = build_warper()
    w.train()
    flow, wl = w(x.float().to(DEV))
    assert flow.shape == flow_ref.shape and len(wl) == len(wl_ref)
    assert rel(flow, flow_ref) < 2e-3
    for a, b in zip(wl, wl_ref):
        assert a.shape == b.shape
        assert abs(float(a.norm()) / float(b.norm()) - 1) < 1e-3
        assert not a.requires_grad
    (flow * rw.float().to(DEV)).sum().backward()
    names = dict(w.named_parameters())
    n = 0
    for k, t in P.items():
        if t.grad is None:
            if k.startswith("connection."):
                assert names[k].grad is None, k   # built but unused: no gradient, as in the reference
            continue
        e, cos = frob(names[k].grad, t.grad)
        assert cos >= 0.999 and e <= 2e-2, (k, e, cos)
        n += 1
    assert n == 43
    sd = w.state_dict()
    for k, t in P.items():
        if "running" in k:
            assert rel(sd[k], t) < 1e-3, k
        if k.endswith("num_batches_tracked"):
            assert int(sd[k]) == 1


def test_warper_rejects_indivisible_input():
    w = build_warper()
    with pytest.raises(ValueError):
        w(torch.zeros(1, 3, 256, 320, device=DEV))


def test_source_only_step_with_warper():
    """train_gta2cityscapes_multi.py:259-286 (SOURCE_ONLY, warper on) vs the oracle."""
    from test_model_gpu import build_g
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    G = R.to_torch(R.det_state(R.g_specs(), 1338), trainable=R.g_trainable)
    W = R.to_torch(R.det_state(RW.warper_specs(), W_SEED, conv_std=W_CONV_STD), trainable=RW.warper_trainable)
    D2 = R.to_torch(R.det_state(R.d_specs(), 2002), trainable=lambda k: True)
    opt, _, _ = R.make_optimizers(G, None, D2, R.DEFAULT_CFG)
    x = torch.from_numpy(R.det_images((2, 3, 256, 256), 21))
    lab = torch.from_numpy(R.det_labels((2, 256, 256), 26))
    g0 = {k: v.detach().clone() for k, v in G.items()}
    ref = RW.source_only_step(G, W, opt, {"input_size": (256, 256)}, 0, [(x, lab)])

    m, w = build_g(), build_warper()
    m.train()
    w.train()
    tr = AdaptSegTrainer(m, None, None, StepConfig(level="source-only", input_size=(256, 256)), warper=w)
    L = tr.step(0, [(x.float().to(DEV), lab.to(DEV))]).values()
    assert abs(L["loss_seg2"] / ref["loss_seg2"] - 1) < 1e-3
    sd = m.state_dict()
    for key in ("conv1.weight", "layer3.5.conv2.weight", "layer4.2.conv3.weight", "layer6.conv2d_list.0.weight"):
        du = (sd[key].detach().double().cpu() - g0[key])
        dr = (G[key].detach() - g0[key])
        assert float(F.cosine_similarity(du.flatten(), dr.flatten(), dim=0)) >= 0.99, key
    wn = dict(w.named_parameters())
    for key in ("encoder_d.down_list.0.input.weight", "decoder_d.up_list.3.block.2.l.weight",
                "decoder_d.up_list.7.output.2.weight", "encoder_d.down_list.4.block.1.norm.weight"):
        _, cos = frob(wn[key].grad, W[key].grad)
        assert cos >= 0.99, (key, cos)
    assert m.layer5.conv2d_list[0].weight.grad is None     # loss_seg2 only: layer5 gets no gradient


def test_single_level_step_with_warper_runs():
    """The single-level step with the warper: the target reuses the source field, detached."""
    from test_model_gpu import build_g, build_d
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    m, d2, w = build_g(), build_d(2002), build_warper()
    m.train()
    w.train()
    tr = AdaptSegTrainer(m, None, d2, StepConfig(level="single-level", input_size=(256, 256),
                                                 input_size_target=(256, 256)), warper=w)
    x = torch.from_numpy(R.det_images((1, 3, 256, 256), 21)).float().to(DEV)
    lab = torch.from_numpy(R.det_labels((1, 256, 256), 26)).to(DEV)
    xt = torch.from_numpy(R.det_images((1, 3, 256, 256), 27)).float().to(DEV)
    L = tr.step(0, [(x, lab, xt)]).values()
    assert all(np.isfinite(v) for v in L.values()) and set(L) == {"loss_seg2", "loss_adv_target2", "loss_D2"}
    assert w.decoder_d.up_list[7].output[2].weight.grad is not None
