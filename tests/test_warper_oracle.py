"""CPU: the warper oracle (oracle/reference_warper.py) against goldens captured from the
reference's own Warper / ResNetMulti.warp / source-only step (tests/golden/gen_warper_golden.py),
and the drop-in module's structure (state_dict keys, shapes, parameter count, init).

Tolerances: fp64 restatement vs fp64 reference, rel 1e-9 (sums and norms of whole tensors
1e-8: host summation order).
"""
import os

import numpy as np
import pytest
import torch

from oracle import reference_torch as R
from oracle import reference_warper as RW

GOLD = os.path.join(os.path.dirname(__file__), "golden", "warper_goldens.npz")
W_SEED, G_SEED, W_CONV_STD = 3001, 1338, 0.02
IMG_SHAPE = (2, 3, 256, 256)
WARP_IN, WARP_FLOW = (2, 19, 16, 24), (2, 2, 16, 24)


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def det_normal(shape, seed, scale=1.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(scale * rng.standard_normal(shape))


def close(a, b, rtol=1e-9, atol=0.0):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    err = np.abs(a - b).max() if a.size else 0.0
    scale = max(np.abs(b).max() if b.size else 0.0, 1e-30)
    assert err <= rtol * scale + atol, (err, scale)


def test_module_keys_shapes_and_param_count():
    from adaptsegnet_amd.model import Warper
    w = Warper()
    sd = w.state_dict()
    specs = RW.warper_specs()
    assert list(sd) == [k for k, _, _ in specs]
    for k, shape, _ in specs:
        assert tuple(sd[k].shape) == tuple(shape), k
    assert sum(p.numel() for p in w.parameters()) == 39161614     # the reference's Warper()
    # init_weights(xavier, gain 0.02) (model/warper.py:182-213): conv weights ~ N(0, std)
    wt = w.decoder_d.up_list[1].block[2].l.weight
    std = 0.02 * np.sqrt(2.0 / (1024 * 9 + 512 * 9))
    assert abs(float(wt.std()) / std - 1) < 0.02
    assert float(w.decoder_d.up_list[7].output[2].bias.abs().max()) == 0.0
    bn = w.encoder_d.down_list[3].block[1].norm
    assert abs(float(bn.weight.mean()) - 1) < 0.01 and float(bn.bias.abs().max()) == 0.0


def test_warper_forward_backward_matches_reference(gold):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    P = R.to_torch(R.det_state(RW.warper_specs(), W_SEED, conv_std=W_CONV_STD), trainable=RW.warper_trainable)
    x = torch.from_numpy(R.det_images(IMG_SHAPE, 21))
    flow, wl = RW.warper_forward(P, x, train=True)
    close(flow.detach()[:, :, ::4, ::4].numpy(), gold["warper/flow_s4"])
    close(flow.detach().sum().item(), gold["warper/flow_sum"], 1e-8, 1e-10)
    close(flow.detach().norm().item(), gold["warper/flow_norm"])
    assert len(wl) == 8
    for i, t in enumerate(wl):
        assert tuple(t.shape) == tuple(gold[f"warper/list{i}_shape"])
        close(t.detach().norm().item(), gold[f"warper/list{i}_norm"])
        close(t.detach().sum().item(), gold[f"warper/list{i}_sum"], 1e-8, 1e-8)
    (flow * det_normal(flow.shape, 22)).sum().backward()
    n = 0
    for k, t in P.items():
        gk = f"warper/gradnorm/{k}"
        if gk in gold:
            close(t.grad.norm().item(), gold[gk], 1e-8)
            n += 1
    assert n == 43      # every trainable parameter but the unused Connection's 12
    for k in ("encoder_d.down_list.0.input.weight", "decoder_d.up_list.7.output.2.weight",
              "decoder_d.up_list.7.output.2.bias"):
        close(P[k].grad.numpy(), gold[f"warper/grad/{k}"], 1e-8)
    for k, t in P.items():
        if "running" in k:
            close(t.sum().item(), gold[f"warper/sum/{k}"], 1e-8, 1e-9)


@pytest.mark.parametrize("tag,scale", [("mod", 0.8), ("sat", 6.0)])
def test_warp_matches_reference(gold, tag, scale):
    inp = det_normal(WARP_IN, 23).requires_grad_(True)
    fl = det_normal(WARP_FLOW, 24, scale).requires_grad_(True)
    out = RW.warp(inp, fl)
    (out * det_normal(out.shape, 25)).sum().backward()
    close(out.detach().numpy(), gold[f"warp_{tag}/out"], 1e-12)
    close(inp.grad.numpy(), gold[f"warp_{tag}/d_input"], 1e-12)
    close(fl.grad.numpy(), gold[f"warp_{tag}/d_flow"], 1e-12)


def test_source_only_step_matches_reference(gold):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    G = R.to_torch(R.det_state(R.g_specs(), G_SEED), trainable=R.g_trainable)
    W = R.to_torch(R.det_state(RW.warper_specs(), W_SEED, conv_std=W_CONV_STD), trainable=RW.warper_trainable)
    D2 = R.to_torch(R.det_state(R.d_specs(), 2002), trainable=lambda k: True)
    opt, _, _ = R.make_optimizers(G, None, D2, R.DEFAULT_CFG)
    x = torch.from_numpy(R.det_images(IMG_SHAPE, 21))
    lab = torch.from_numpy(R.det_labels((IMG_SHAPE[0], IMG_SHAPE[2], IMG_SHAPE[3]), 26))
    cfg = {"input_size": (IMG_SHAPE[3], IMG_SHAPE[2])}
    for it in range(2):
        v = RW.source_only_step(G, W, opt, cfg, it, [(x, lab)])
        close(v["loss_seg2"], gold[f"source_only/loss_seg2/{it}"], 1e-9)
    for k, t in G.items():
        if f"source_only/sum/{k}" in gold:
            close(t.detach().double().sum().item(), gold[f"source_only/sum/{k}"], 1e-8, 1e-8)
            close(t.detach().double().norm().item(), gold[f"source_only/norm/{k}"], 1e-9)
    n = 0
    for k, t in W.items():
        gk = f"source_only/warper_gradnorm/{k}"
        if gk in gold:
            close(t.grad.norm().item(), gold[gk], 1e-7)
            n += 1
    assert n == 43
