"""Deferred split-K sums of weight gradients (adaptseg.h ADAPTSEG_WGRAD_DEFER_SUM,
adaptseg_splitk_flush; engine.DEFER_SPLITK): the sums a weight gradient leaves pending run at
the flush, in issue order, and give bitwise the immediate sums' gradients — per product, for
several products accumulating into one gradient, for products that do not split K (written
directly), and over whole training steps.  Reference call sites: the weight gradients autograd
computes for every nn.Conv2d of model/deeplab_multi.py / discriminator.py in
train_gta2cityscapes_multi.py:437-462 / 626-679 (loss.backward())."""
import pytest
import torch

from test_x3_terms_gpu import nhwc, w_cl

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def k():
    from adaptsegnet_amd import kernels
    return kernels


# (n, cin, h, w, cout, ks, stride, pad, dil)
SHAPES = [
    (2, 256, 24, 40, 256, 3, 1, 2, 2),      # layer3 conv2 class (term-image / x3h weight gradient)
    (2, 1024, 16, 24, 256, 1, 1, 0, 1),     # conv1 (staged weight gradient, many splits)
    (2, 64, 40, 44, 128, 3, 1, 1, 1),       # layer2-class 3x3
    (1, 64, 97, 131, 64, 3, 1, 1, 1),       # odd sizes
]


def _operands(shape, seed):
    n, cin, h, w, cout, ks, stride, pad, dil = shape
    g = torch.Generator().manual_seed(seed)
    from adaptsegnet_amd import kernels
    geom = kernels.ConvGeom(cin, cout, ks, ks, stride, (pad,), (dil,))
    oh, ow = geom.out_hw(h, w)
    x = nhwc(torch.randn(n, cin, h, w, generator=g))
    gy = nhwc(torch.randn(n, cout, oh, ow, generator=g))
    w0 = w_cl(torch.randn(cout, cin, ks, ks, generator=g))
    return geom, x, gy, w0


@pytest.mark.parametrize("shape", SHAPES, ids=[f"s{i}" for i in range(len(SHAPES))])
def test_deferred_sum_is_bitwise_the_immediate_one(k, shape):
    n, cin, h, w = shape[0], shape[1], shape[2], shape[3]
    geom, x, gy, w0 = _operands(shape, 5)
    _, splits = k.conv_kernel_id(geom, n, h, w, 2)
    dw_imm, dw_def = w0.clone(), w0.clone()
    k.conv_wgrad(geom, gy, x, n, h, w, [dw_imm])
    assert k.splitk_pending() == 0
    k.conv_wgrad(geom, gy, x, n, h, w, [dw_def], defer=True)
    assert k.splitk_pending() == (1 if splits > 1 else 0), splits
    if splits > 1:
        torch.cuda.synchronize()
        assert torch.equal(dw_def, w0)   # nothing written into dw before the flush
    k.splitk_flush()
    assert k.splitk_pending() == 0
    assert torch.equal(dw_imm, dw_def)


def test_deferred_sums_keep_issue_order(k):
    """Three products into one gradient (two split, one not) and one into another: the flush
    adds in issue order, so the results equal the immediate sequence bitwise."""
    shape = SHAPES[0]
    n, h, w = shape[0], shape[2], shape[3]
    geom, x, gy, w0 = _operands(shape, 9)
    _, x2, gy2, _ = _operands(shape, 10)
    s1 = SHAPES[1]
    geom1, x1, gy1, w1 = _operands(s1, 11)
    a_imm, a_def, b_imm, b_def = w0.clone(), w0.clone(), w1.clone(), w1.clone()
    for defer, a, b in ((False, a_imm, b_imm), (True, a_def, b_def)):
        k.conv_wgrad(geom, gy, x, n, h, w, [a], defer=defer)
        k.conv_wgrad(geom1, gy1, x1, s1[0], s1[2], s1[3], [b], defer=defer)
        k.conv_wgrad(geom, gy2, x2, n, h, w, [a], defer=defer)
    assert k.splitk_pending() >= 2
    k.splitk_flush()
    assert torch.equal(a_imm, a_def) and torch.equal(b_imm, b_def)


def test_flush_is_per_stream(k):
    """A sum deferred on one stream is not launched by another stream's flush."""
    shape = SHAPES[1]
    n, h, w = shape[0], shape[2], shape[3]
    geom, x, gy, w0 = _operands(shape, 13)
    assert k.conv_kernel_id(geom, n, h, w, 2)[1] > 1
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    dw = w0.clone()
    with torch.cuda.stream(side):
        k.conv_wgrad(geom, gy, x, n, h, w, [dw], defer=True)
        assert k.splitk_pending() == 1
    assert k.splitk_pending() == 0   # the default stream has none
    k.splitk_flush()                 # ... so this launches nothing
    with torch.cuda.stream(side):
        assert k.splitk_pending() == 1
        k.splitk_flush()
    torch.cuda.current_stream().wait_stream(side)
    ref = w0.clone()
    k.conv_wgrad(geom, gy, x, n, h, w, [ref])
    assert torch.equal(ref, dw)


def test_training_steps_bit_identical_with_deferred_sums(monkeypatch):
    """engine.DEFER_SPLITK 1 vs 0 (the default): the same losses and parameters, bit for bit,
    over two multi-level LS steps with iter_size 2 (both generator backwards and the
    discriminators' defer, flush at their joins)."""
    from adaptsegnet_amd import engine
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    from test_model_gpu import R, build_d, build_g
    shape_s, shape_t = (1, 3, 41, 57), (1, 3, 33, 49)
    subs = [(torch.from_numpy(R.det_images(shape_s, 41 + i)).float().to(DEV),
             torch.from_numpy(R.det_labels((1, 41, 57), 42 + i)).to(DEV),
             torch.from_numpy(R.det_images(shape_t, 43 + i)).float().to(DEV)) for i in (0, 10)]
    cfg = dict(level="multi-level", gan="LS", input_size=(57, 41), input_size_target=(49, 33), iter_size=2)
    runs = []
    for defer in (1, 0):
        monkeypatch.setattr(engine, "DEFER_SPLITK", defer)
        m, d1, d2 = build_g(), build_d(2001), build_d(2002)
        m.train()
        tr = AdaptSegTrainer(m, d1, d2, StepConfig(**cfg))
        losses = [tr.step(it, subs).values() for it in range(2)]
        torch.cuda.synchronize()
        runs.append((losses, [{kk: v.detach().cpu().clone() for kk, v in mm.state_dict().items()}
                              for mm in (m, d1, d2)]))
    (l0, s0), (l1, s1) = runs
    assert l0 == l1
    for a, b in zip(s0, s1):
        for kk in a:
            assert torch.equal(a[kk], b[kk]), kk
