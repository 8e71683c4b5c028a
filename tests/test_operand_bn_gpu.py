"""Operand BatchNorm (adaptseg.h adaptseg_operand_bn; engine.BN_FOLD): a train-mode BN + ReLU folded
into its consumer conv's operand gather — the x3h forward (with the fused output statistics) and
the register-staged F32X3 weight gradient read the BN's input and apply the BN themselves.  The
results must equal the unfused chain (BN apply pass, then the conv on its output) BIT FOR BIT:
the same expression (common.hpp bn_relu), the same products, the same plans.  Reference:
model/deeplab_multi.py:92-95 (out = relu(bn2(conv2(out))); out = conv3(out)) in the train step
train_gta2cityscapes_multi.py:385-461."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def k():
    from adaptsegnet_amd import kernels
    return kernels


# producer conv (Cin0 -> C, ks0) feeding the BN, then the consumer (C -> Cout, ks, pad, dil)
# (n, cin0, h, w, c, cout, ks, pad, dil)
CASES = [
    (2, 64, 96, 96, 512, 1024, 1, 0, 1),    # a 512-channel BN into a 1x1 (the x3h forward needs K >= 512)
    (2, 128, 96, 96, 512, 2048, 1, 0, 1),   # layer4 class
    (4, 64, 96, 96, 256, 256, 3, 2, 2),     # a dilated 3x3 consumer: padding taps read 0, not relu(b)
    (2, 64, 97, 89, 512, 512, 1, 0, 1),     # odd sizes: ragged row tiles / K tail of the weight gradient
]


def _chain(k, case, seed):
    n, cin0, h, w, c, cout, ks, pad, dil = case
    g = torch.Generator().manual_seed(seed)
    g0 = k.ConvGeom(cin0, c, 1, 1, 1, (0,), (1,))
    g1 = k.ConvGeom(c, cout, ks, ks, 1, (pad,), (dil,))
    x0 = torch.randn(n, h, w, cin0, generator=g).to(DEV)
    w0 = (torch.randn(c, 1, 1, cin0, generator=g) / cin0 ** 0.5).to(DEV)
    w1 = (torch.randn(cout, ks, ks, c, generator=g) / (c * ks * ks) ** 0.5).to(DEV)
    bnw = (1 + 0.2 * torch.randn(c, generator=g)).to(DEV)
    bnb = (0.2 * torch.randn(c, generator=g)).to(DEV)
    xp, tiles = k.conv_fwd_bnstats(g0, x0, n, h, w, [w0])
    assert tiles is not None
    return g1, xp, tiles, w1, bnw, bnb


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
def test_operand_bn_is_bitwise_the_unfused_chain(k, case):
    n, _, h, w, c, cout, ks, _, _ = case
    g1, xp, tiles, w1, bnw, bnb = _chain(k, case, 17 + case[4])
    assert k.operand_bn_ok(g1, n, h, w, 0) and k.operand_bn_ok(g1, n, h, w, 2)
    rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
    y, mean, invstd = k.bn_fwd_train_tiles(xp, tiles, bnw, bnb, rm.clone(), rv.clone(), 0.1, 1e-5)
    rm2, rv2 = rm.clone(), rv.clone()
    m2, i2 = k.bn_fwd_train_tiles_stats(xp, tiles, rm2, rv2, 0.1, 1e-5)
    assert torch.equal(m2, mean) and torch.equal(i2, invstd)
    rm1, rv1 = rm.clone(), rv.clone()
    k.bn_fwd_train_tiles(xp, tiles, bnw, bnb, rm1, rv1, 0.1, 1e-5)
    assert torch.equal(rm1, rm2) and torch.equal(rv1, rv2)   # the running statistics too
    abn = k.OperandBN(mean, invstd, bnw, bnb)
    # forward with the fused output statistics
    y3, t3 = k.conv_fwd_bnstats(g1, y, n, h, w, [w1])
    z3, u3 = k.conv_fwd_bnstats_abn(g1, xp, abn, n, h, w, [w1])
    assert t3 is not None and t3[1] == u3[1]
    assert torch.equal(y3, z3)
    assert torch.equal(t3[0], u3[0])
    # weight gradient, accumulated into an existing gradient
    oh, ow = g1.out_hw(h, w)
    gg = torch.Generator().manual_seed(5)
    dy = torch.randn(n, oh, ow, cout, generator=gg).to(DEV)
    dw0 = torch.randn(cout, ks, ks, c, generator=gg).to(DEV)
    dwa, dwb = dw0.clone(), dw0.clone()
    k.conv_wgrad(g1, dy, y, n, h, w, [dwa])
    k.conv_wgrad_abn(g1, dy, xp, abn, n, h, w, [dwb])
    assert torch.equal(dwa, dwb)
    # and the fused forward against fp64 (BN + ReLU + conv)
    yd = torch.relu((xp.double() - mean.double()) * invstd.double() * bnw.double() + bnb.double())
    ref = torch.nn.functional.conv2d(yd.permute(0, 3, 1, 2).cpu(), w1.double().permute(0, 3, 1, 2).cpu(), None, 1,
                                     case[7], case[8])
    got = z3.permute(0, 3, 1, 2).double().cpu()
    assert float((got - ref).abs().max() / ref.abs().max()) < 2e-5


def test_operand_bn_eligibility(k):
    # the x3h forward needs K >= 512 and a BN of <= 512 channels
    assert not k.operand_bn_ok(k.ConvGeom(256, 1024, 1, 1, 1, (0,), (1,)), 2, 64, 64, 0)  # K 256: staged forward
    assert not k.operand_bn_ok(k.ConvGeom(1024, 256, 1, 1, 1, (0,), (1,)), 2, 64, 64, 0)  # C 1024 > 512
    assert k.operand_bn_ok(k.ConvGeom(512, 2048, 1, 1, 1, (0,), (1,)), 2, 64, 64, 0)
    assert k.operand_bn_ok(k.ConvGeom(256, 256, 3, 3, 1, (2,), (2,)), 4, 96, 96, 0)      # K 2304


def test_training_steps_bit_identical_with_folded_bn(monkeypatch):
    """engine.BN_FOLD 3 (BN2 -> conv3 and BN1 -> conv2) vs 0 (the default) over two single-level
    steps at the c2 bench shape (batch 4, 1024x512: the producing convs' unsplit plans carry the
    statistics tiles the fold needs; layer 4 folds BN2 (layer 3's conv3 has K 256: staged), layers 1
    and 3 BN1 — layer 4's conv2 keeps its
    term-image weight gradient, X3_WGRAD_TERMS_MIN_C — counted): the same
    losses and parameters, bit for bit."""
    from adaptsegnet_amd import engine
    from adaptsegnet_amd import kernels as K
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    from test_model_gpu import R, build_d, build_g
    shape = (4, 3, 512, 1024)
    batch = [(torch.from_numpy(R.det_images(shape, 61)).float().to(DEV),
              torch.from_numpy(R.det_labels((4, 512, 1024), 62)).to(DEV),
              torch.from_numpy(R.det_images(shape, 63)).float().to(DEV))]
    cfg = dict(level="single-level", gan="Vanilla", input_size=(1024, 512), input_size_target=(1024, 512))
    calls = []
    orig = K.conv_fwd_bnstats_abn

    def counting(*a, **kw):
        calls.append(1)
        return orig(*a, **kw)
    monkeypatch.setattr(K, "conv_fwd_bnstats_abn", counting)
    runs = []
    for fold in (3, 0):
        monkeypatch.setattr(engine, "BN_FOLD", fold)
        calls.clear()
        m, d2 = build_g(), build_d(2002)
        m.train()
        tr = AdaptSegTrainer(m, None, d2, StepConfig(**cfg))
        losses = [tr.step(it, batch).values() for it in range(2)]
        torch.cuda.synchronize()
        if fold:
            assert len(calls) >= 2 * 3 + 2 * 26   # BN2 of layer 4, BN1 of layers 1, 3; per step
        else:
            assert not calls
        runs.append((losses, [{kk: v.detach().cpu().clone() for kk, v in mm.state_dict().items()}
                              for mm in (m, d2)]))
    (l0, s0), (l1, s1) = runs
    assert l0 == l1
    for a, b in zip(s0, s1):
        for kk in a:
            assert torch.equal(a[kk], b[kk]), kk
