"""igemm_x3h_kernel (conv_x3r.hpp, selectors 100*op + 86 / 87): the 256x128x32 F32X3 tile with the
fp32 activation operand split in-kernel, and igemm_x3hw_kernel<128> (selector 287), the 128-row
weight-gradient tile with both fp32 operands split in-kernel (adaptseg_conv_set_x3h / ADAPTSEG_X3H).

Same six products, per-accumulator k order and epilogue as the term-image kernel (selectors 88 /
89) — only the operand path differs (register-gathered fp32 rows split while staged instead of
LDS-DMA of pre-split term images) — so a product equals the term-image kernel's BITWISE on the
same plan, and the fp64 oracle at the conv parity tolerance (2e-5 * max|ref|).  Covered: the
Bottleneck / downsample / DeeplabVGG shape classes (dilated 3x3, 1x1 narrowing / widening, the
stride-2 1x1 downsample and its parity-class data gradient, odd sizes with grid tails, split-K
grids), the fused BN statistics, bias + ReLU, the residual / ReLU' / accumulate epilogues and
the term-image outputs.  Reference call sites: model/deeplab_multi.py:59-103 (Bottleneck),
:106-121 (Classifier_Module), model/deeplab_vgg.py:34-43.
"""
import pytest
import torch
import torch.nn.functional as F

from test_x3_terms_gpu import nchw, nhwc, rel, terms, w_cl

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def k():
    from adaptsegnet_amd import kernels
    old = kernels.get_x3h()
    kernels.set_x3h(7)
    yield kernels
    kernels.set_x3h(old)


def x3h_eligible(cin, cout, ks, stride, op):
    """The library's x3h rule (conv_igemm.hip make_plan): K >= 512 (ADAPTSEG_X3H_MIN_K), no
    stride-2 data gradient."""
    return ks * ks * (cin if op == 0 else cout) >= 512 and not (op == 1 and stride == 2)


# (n, cin, h, w, cout, ks, stride, pad, dil)
SHAPES = [
    (2, 256, 24, 40, 256, 3, 1, 2, 2),      # layer3 conv2 (dilated 3x3)
    (2, 512, 20, 24, 512, 3, 1, 4, 4),      # layer4 conv2
    (2, 1024, 16, 24, 256, 1, 1, 0, 1),     # conv1 (narrowing 1x1)
    (2, 256, 16, 24, 1024, 1, 1, 0, 1),     # conv3 (widening 1x1)
    (2, 256, 30, 34, 512, 1, 2, 0, 1),      # layer2 downsample (stride-2 1x1: parity-class dgrad)
    (2, 64, 40, 44, 128, 3, 1, 1, 1),       # layer2-class 3x3, Cin 64 (two 32-deep steps per tap)
    (1, 64, 97, 131, 64, 3, 1, 1, 1),       # layer1 conv2, odd sizes (grid tails)
    (4, 256, 128, 128, 256, 1, 1, 0, 1),    # >= 256 tiles: unsplit, in-kernel epilogue
    (2, 128, 34, 62, 256, 4, 2, 1, 1),      # discriminator 4x4 / 2 (its data gradient: parity classes)
    (4, 64, 80, 96, 256, 1, 1, 0, 1),       # layer1 conv3 (K 64: the register-staged forward)
]


@pytest.mark.parametrize("shape", SHAPES, ids=[f"s{i}" for i in range(len(SHAPES))])
def test_x3h_matches_term_kernel_bitwise_and_fp64(k, shape):
    n, cin, h, w, cout, ks, stride, pad, dil = shape
    geom = k.ConvGeom(cin, cout, ks, ks, stride, (pad,), (dil,))
    oh, ow = geom.out_hw(h, w)
    g = torch.Generator().manual_seed(hash(shape) % 1000 + 7)
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, ks, ks, generator=g, dtype=torch.float64) / (cin * ks * ks) ** 0.5
    gy = torch.randn(n, cout, oh, ow, generator=g, dtype=torch.float64)
    xd, gyd, wd = nhwc(x), nhwc(gy), w_cl(wt)
    same = {}
    for op in (0, 1):
        sel_h, sp_h = k.conv_kernel_id(geom, n, h, w, op)
        sel_t, sp_t = k.conv_kernel_id(geom, n, h, w, op, copies=True)
        assert sel_t % 100 in (88, 89), (op, sel_t)
        if x3h_eligible(cin, cout, ks, stride, op):
            assert sel_h % 100 in (86, 87), (op, sel_h)
            assert sel_h % 100 - 86 == sel_t % 100 - 88 and sp_h == sp_t   # the same plan
            same[op] = True
        else:   # K < 512 or a stride-2 data gradient: the register-staged kernel
            assert sel_h % 100 in (95, 96), (op, sel_h)
            same[op] = sp_h == 1 and sp_t == 1   # unsplit: bitwise equal as well
    ref = F.conv2d(x, wt, None, stride, pad, dil)
    y_h = k.conv_fwd(geom, xd, n, h, w, [wd])
    y_t = k.conv_fwd(geom, None, n, h, w, [wd], xb=terms(xd))
    assert rel(nchw(y_h), ref) < 2e-5
    if same[0]:
        assert torch.equal(y_h, y_t)
    dref = torch.nn.grad.conv2d_input(x.shape, wt, gy, stride, pad, dil)
    dx_h = k.conv_dgrad(geom, gyd, n, h, w, [wd])
    dx_t = k.conv_dgrad(geom, None, n, h, w, [wd], dyb=terms(gyd))
    assert rel(nchw(dx_h), dref) < 2e-5
    if same[1]:
        assert torch.equal(dx_h, dx_t)
    # weight gradient (igemm_x3hw_kernel<128>), accumulated into an existing gradient
    sel_w, sp_w = k.conv_kernel_id(geom, n, h, w, 2)
    sel_wt, sp_wt = k.conv_kernel_id(geom, n, h, w, 2, copies=True)
    assert sel_w == 287 and sel_wt in (288, 289), (sel_w, sel_wt)
    w0 = torch.randn(cout, cin, ks, ks, generator=g, dtype=torch.float64)
    wref = torch.nn.grad.conv2d_weight(x, wt.shape, gy, stride, pad, dil) + w0
    dw_h, dw_t = w_cl(w0), w_cl(w0)
    k.conv_wgrad(geom, gyd, xd, n, h, w, [dw_h])
    k.conv_wgrad(geom, None, None, n, h, w, [dw_t], dyb=terms(gyd), xb=terms(xd))
    assert rel(dw_h.permute(0, 3, 1, 2), wref) < 2e-5
    if sel_wt == 289 and sp_wt == sp_w:   # the same plan: the same products in the same order
        assert torch.equal(dw_h, dw_t)


def test_x3h_mode_bits_select_the_kernels(k):
    geom = k.ConvGeom(256, 256, 3, 3, 1, (2,), (2,))
    sels = lambda: [k.conv_kernel_id(geom, 2, 24, 40, op)[0] for op in (0, 1, 2)]  # noqa: E731
    k.set_x3h(0)
    assert sels() == [95, 195, 295]
    k.set_x3h(1)
    assert sels() == [86, 195, 295]
    k.set_x3h(2)
    assert sels() == [95, 186, 295]
    k.set_x3h(4)
    assert sels() == [95, 195, 287]


def test_x3h_fused_bn_statistics(k):
    """conv_fwd_bnstats on the x3h tile: 256-row statistics tiles, bitwise the term kernel's."""
    n, cin, h, w, cout = 2, 256, 128, 128, 256
    geom = k.ConvGeom(cin, cout, 3, 3, 1, (2,), (2,))
    g = torch.Generator().manual_seed(11)
    xd = nhwc(torch.randn(n, cin, h, w, generator=g))
    wd = w_cl(torch.randn(cout, cin, 3, 3, generator=g) / 48)
    y0, t0 = k.conv_fwd_bnstats(geom, xd, n, h, w, [wd])
    y1, t1 = k.conv_fwd_bnstats(geom, None, n, h, w, [wd], xb=terms(xd))
    assert t0 is not None and t1 is not None and t0[1] == t1[1]
    assert torch.equal(y0, y1)
    bw, bb = torch.ones(cout, device=DEV), torch.zeros(cout, device=DEV)
    _, m0, i0 = k.bn_fwd_train_tiles(y0, t0, bw, bb, None, None, 0.1, 1e-5)
    _, m1, i1 = k.bn_fwd_train_tiles(y1, t1, bw, bb, None, None, 0.1, 1e-5)
    assert torch.equal(m0, m1) and torch.equal(i0, i1)


# (n, cin, h, w, cout, k, stride, pad, dil, bias)
EPI_SHAPES = [(1, 64, 9, 11, 64, 3, 1, 1, 1, True), (2, 128, 48, 64, 128, 3, 1, 1, 1, True),
              (2, 64, 20, 24, 128, 1, 2, 0, 1, False), (4, 256, 64, 64, 512, 1, 1, 0, 1, False)]


@pytest.mark.parametrize("shape", EPI_SHAPES, ids=[f"e{i}" for i in range(len(EPI_SHAPES))])
def test_x3h_epilogues(k, shape):
    """bias + ReLU (DeeplabVGG), the term-image outputs, the ReLU' / residual / accumulate data
    gradients: bitwise the term-image kernel's, and the fp64 oracle within 2e-5."""
    n, cin, h, w, cout, ks, st, pd, dl, bias = shape
    g = torch.Generator().manual_seed(78)
    x = torch.randn(n, h, w, cin, generator=g).to(DEV)
    wt = (torch.randn(cout, ks, ks, cin, generator=g) * 0.1).to(DEV)
    b = torch.randn(cout, generator=g).to(DEV) if bias else None
    geo = k.ConvGeom(cin, cout, ks, ks, st, (pd,), (dl,))
    oh, ow = geo.out_hw(h, w)
    y, yt = k.conv_fwd(geo, x, n, h, w, [wt], [b] if bias else None, flags=k.EPI_RELU, bf16_out=True)
    y2, yt2 = k.conv_fwd(geo, None, n, h, w, [wt], [b] if bias else None, flags=k.EPI_RELU, bf16_out=True,
                         xb=terms(x))
    assert torch.equal(yt, terms(y)) and torch.equal(y, y2) and torch.equal(yt, yt2)
    ref = F.relu(F.conv2d(x.permute(0, 3, 1, 2).double().cpu(), wt.permute(0, 3, 1, 2).double().cpu(),
                          b.double().cpu() if bias else None, st, pd, dl))
    assert rel(nchw(y), ref) < 2e-5
    dy = torch.randn(n, oh, ow, cout, generator=g).to(DEV)
    aux = F.relu(torch.randn(n, h, w, cin, generator=g)).to(DEV)
    dx, dxt = k.conv_dgrad(geo, dy, n, h, w, [wt], aux=aux, flags=k.EPI_RELU_GRAD, bf16_out=True)
    dx2, dxt2 = k.conv_dgrad(geo, None, n, h, w, [wt], aux=aux, flags=k.EPI_RELU_GRAD, bf16_out=True,
                             dyb=terms(dy))
    assert torch.equal(dxt, terms(dx)) and torch.equal(dx, dx2) and torch.equal(dxt, dxt2)
    res = torch.randn(n, h, w, cin, generator=g).to(DEV)
    dx3 = k.conv_dgrad(geo, dy, n, h, w, [wt], res=res)
    dx4 = k.conv_dgrad(geo, None, n, h, w, [wt], res=res, dyb=terms(dy))
    assert torch.equal(dx3, dx4)
    dref = torch.nn.grad.conv2d_input((n, cin, h, w), wt.permute(0, 3, 1, 2).double().cpu(),
                                      dy.permute(0, 3, 1, 2).double().cpu(), st, pd, dl)
    assert rel(nchw(dx3), dref + res.permute(0, 3, 1, 2).double().cpu()) < 2e-5
