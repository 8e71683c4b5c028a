"""F32X3 operand copies: the three exact bf16 term images of an fp32 activation.

Under the default F32X3 conv math the BatchNorm passes that produce conv operands write, beside
(or instead of) the fp32 tensor, its three bf16 terms, pixel-interleaved [..., 3, C] (hi + mid +
lo == v exactly for |v| >= 2^-126, each the RNE bf16 of what is left: common.hpp split3), and the
Bottleneck convs read them through
the 256x128x32 LDS-DMA kernel (conv_x3r.hpp, selectors 100*op + 88 / 89) instead of splitting
fp32 rows in-kernel (conv_x3.hpp).  Checked here:
  * the BN passes write exactly torch's RNE split, and read terms (residual, ReLU-mask source)
    as the exact fp32 value (bitwise the fp32-storage results);
  * a conv on the terms runs the term-image kernel and equals the register-staged F32X3 kernel
    BITWISE when neither splits K (same six products, same per-accumulator k order), and the
    fp64 oracle at the conv parity tolerance (2e-5 * max|ref|) always — fused BN statistics,
    the stride-2 parity path and 128-row weight gradients included.
Reference call sites: model/deeplab_multi.py:83-103 (Bottleneck: conv -> BN -> ReLU -> conv).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def K():
    from adaptsegnet_amd import kernels
    return kernels


def terms(t):
    """torch's three-term RNE split of an fp32 tensor [..., C] -> its pixel-interleaved copy
    [..., 3, C] bf16 (bn.hip x3_off)."""
    hi = t.to(torch.bfloat16)
    r = t - hi.float()
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    return torch.stack([hi, mid, lo], dim=-2)


def join(tb):
    return (tb[..., 0, :].float() + tb[..., 1, :].float()) + tb[..., 2, :].float()


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous().float().to(DEV)


def nchw(t):
    return t.permute(0, 3, 1, 2).double().cpu()


def w_cl(w):
    return w.permute(0, 2, 3, 1).contiguous().float().to(DEV)


def test_engine_writes_term_copies_only_under_presplit():
    """F32X3 (default): the engine passes no copies (register-staged kernels); F32X3_PRESPLIT:
    the BN passes write term copies and the Bottleneck convs read them."""
    k = K()
    from adaptsegnet_amd import engine
    assert k.get_conv_math() == k.MATH_F32X3 and k.copies_are_terms()
    assert not engine.bf16_operands() and not engine.lowp_storage()
    k.set_conv_math(k.MATH_F32X3_PRESPLIT)
    try:
        assert engine.bf16_operands() and not engine.lowp_storage()
    finally:
        k.set_conv_math(k.MATH_F32X3)


@pytest.mark.parametrize("relu", [0, 1])
def test_bn_forward_writes_and_reads_exact_terms(relu):
    k = K()
    g = torch.Generator().manual_seed(3)
    rows, c = 3 * 37 * 29, 96
    x = torch.randn(rows, c, generator=g).to(DEV) * 3 + 1
    res = torch.randn(rows, c, generator=g).to(DEV)
    w, b = torch.rand(c, generator=g).to(DEV) + 0.5, torch.randn(c, generator=g).to(DEV)
    rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
    # fp32 residual, fp32 output + its terms
    y, mean, invstd, yb = k.bn_fwd_train(x, w, b, rm.clone(), rv.clone(), 0.1, 1e-5, res=res, relu=bool(relu),
                                         bf16_out=True)
    assert yb.shape == (rows, 3, c) and yb.dtype == torch.bfloat16
    assert torch.equal(yb, terms(y)) and torch.equal(join(yb), y)
    # the residual as terms only: bitwise the same output
    y2, _, _, yb2 = k.bn_fwd_train(x, w, b, rm.clone(), rv.clone(), 0.1, 1e-5, res=terms(res),
                                   relu=bool(relu), bf16_out=True, fp32_out=False)
    assert y2 is None and torch.equal(yb2, yb)
    # eval-mode BN on the same storage
    yi = k.bn_fwd_infer(x, w, b, rm, rv, 1e-5, res=res, relu=bool(relu))
    yi2, ybi = k.bn_fwd_infer(x, w, b, rm, rv, 1e-5, res=terms(res), relu=bool(relu), bf16_out=True)
    assert torch.equal(yi2, yi) and torch.equal(ybi, terms(yi))


def test_bn_backward_reads_mask_terms_and_writes_dx_terms():
    k = K()
    g = torch.Generator().manual_seed(5)
    rows, c = 2 * 33 * 41, 128
    x = torch.randn(rows, c, generator=g).to(DEV)
    res = torch.randn(rows, c, generator=g).to(DEV)
    w, b = torch.rand(c, generator=g).to(DEV) + 0.5, torch.randn(c, generator=g).to(DEV)
    y, mean, invstd = k.bn_fwd_train(x, w, b, None, None, 0.1, 1e-5, res=res, relu=True)
    dy = torch.randn(rows, c, generator=g).to(DEV)
    dx, dxb = k.bn_bwd(dy, y, x, w, mean, invstd, relu=True, dres=None, bias=b, bf16_out=True)
    assert dxb.shape == (rows, 3, c) and torch.equal(dxb, terms(dx))
    dx2, dxb2 = k.bn_bwd(dy, terms(y), x, w, mean, invstd, relu=True, bias=b, bf16_out=True)
    assert torch.equal(dx2, dx) and torch.equal(dxb2, dxb)
    # eval mode: mask from the saved output's terms
    e1 = k.bn_bwd(dy, y, None, w, None, invstd, relu=True, train=False)
    e2 = k.bn_bwd(dy, terms(y), None, w, None, invstd, relu=True, train=False)
    assert torch.equal(e1, e2)


# (n, cin, h, w, cout, ks, stride, pad, dil): the Bottleneck / downsample shape classes
SHAPES = [
    (2, 256, 24, 40, 256, 3, 1, 2, 2),      # layer3 conv2 (dilated 3x3)
    (2, 512, 20, 24, 512, 3, 1, 4, 4),      # layer4 conv2
    (2, 1024, 16, 24, 256, 1, 1, 0, 1),     # conv1 (narrowing 1x1)
    (2, 256, 16, 24, 1024, 1, 1, 0, 1),     # conv3 (widening 1x1)
    (2, 256, 30, 34, 512, 1, 2, 0, 1),      # layer2 downsample (stride-2 1x1: parity-class dgrad)
    (2, 64, 40, 44, 128, 3, 1, 1, 1),       # Cout < 256: 128-row weight-gradient tiles
    (1, 64, 97, 131, 64, 3, 1, 1, 1),       # layer1 conv2, odd sizes (grid tails)
]


@pytest.mark.parametrize("shape", SHAPES, ids=[f"s{i}" for i in range(len(SHAPES))])
def test_conv_on_terms_matches_staged_kernel_and_fp64(shape):
    k = K()
    n, cin, h, w, cout, ks, stride, pad, dil = shape
    geom = k.ConvGeom(cin, cout, ks, ks, stride, (pad,), (dil,))
    oh, ow = geom.out_hw(h, w)
    g = torch.Generator().manual_seed(hash(shape) % 1000)
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, ks, ks, generator=g, dtype=torch.float64) / (cin * ks * ks) ** 0.5
    gy = torch.randn(n, cout, oh, ow, generator=g, dtype=torch.float64)
    xd, gyd, wd = nhwc(x), nhwc(gy), w_cl(wt)
    xt, gyt = terms(xd), terms(gyd)
    for op in (0, 1, 2):
        sel_t, sp_t = k.conv_kernel_id(geom, n, h, w, op, copies=True)
        sel_s, sp_s = k.conv_kernel_id(geom, n, h, w, op)
        # without copies: the register-staged kernel, or (ADAPTSEG_OPT_X3H, K >= 256) the same
        # 256x128x32 tile splitting fp32 rows in-kernel
        assert sel_t % 100 in (88, 89) and sel_s % 100 in (86, 87, 95, 96), (op, sel_t, sel_s)
    # forward
    ref = F.conv2d(x, wt, None, stride, pad, dil)
    y_s = k.conv_fwd(geom, xd, n, h, w, [wd])
    y_t = k.conv_fwd(geom, None, n, h, w, [wd], xb=xt)
    assert rel(nchw(y_t), ref) < 2e-5
    if k.conv_kernel_id(geom, n, h, w, 0, copies=True)[1] == 1 and k.conv_kernel_id(geom, n, h, w, 0)[1] == 1:
        assert torch.equal(y_t, y_s)
    # data gradient
    dref = torch.nn.grad.conv2d_input(x.shape, wt, gy, stride, pad, dil)
    dx_s = k.conv_dgrad(geom, gyd, n, h, w, [wd])
    dx_t = k.conv_dgrad(geom, None, n, h, w, [wd], dyb=gyt)
    assert rel(nchw(dx_t), dref) < 2e-5
    if k.conv_kernel_id(geom, n, h, w, 1, copies=True)[1] == 1 and k.conv_kernel_id(geom, n, h, w, 1)[1] == 1:
        assert torch.equal(dx_t, dx_s)
    # weight gradient (accumulate into an existing gradient, as the arena does)
    w0 = torch.randn(cout, cin, ks, ks, generator=g, dtype=torch.float64)
    wref = torch.nn.grad.conv2d_weight(x, wt.shape, gy, stride, pad, dil) + w0
    dw = w_cl(w0)
    k.conv_wgrad(geom, None, None, n, h, w, [dw], dyb=gyt, xb=xt)
    assert rel(dw.permute(0, 3, 1, 2), wref) < 2e-5


def test_fused_bn_statistics_on_terms():
    """conv_fwd_bnstats with x's terms: 256-row statistics tiles (the host query plans them),
    merged by the BN into the same batch statistics as the fp32 path (to fp32 rounding)."""
    k = K()
    n, cin, h, w, cout = 2, 256, 128, 128, 256   # >= 256 tiles of 256 rows: no K split
    geom = k.ConvGeom(cin, cout, 3, 3, 1, (2,), (2,))
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) / 48
    xd, wd = nhwc(x), w_cl(wt)
    y0, t0 = k.conv_fwd_bnstats(geom, xd, n, h, w, [wd])
    y1, t1 = k.conv_fwd_bnstats(geom, None, n, h, w, [wd], xb=terms(xd))
    # 128-row tiles on the register-staged kernel, 256 on the x3h one (the default here, K 2304)
    rows0 = 256 if k.conv_kernel_id(geom, n, h, w, 0)[0] % 100 == 86 else 128
    assert t0 is not None and t1 is not None and t1[1] * 256 // rows0 == t0[1]
    assert torch.equal(y0, y1)   # neither splits K: bitwise the staged kernel
    bw, bb = torch.ones(cout, device=DEV), torch.zeros(cout, device=DEV)
    _, m0, i0 = k.bn_fwd_train_tiles(y0, t0, bw, bb, None, None, 0.1, 1e-5)
    _, m1, i1 = k.bn_fwd_train_tiles(y1, t1, bw, bb, None, None, 0.1, 1e-5)
    ref = y0.double().reshape(-1, cout)
    assert rel(m1, ref.mean(0)) < 1e-5 and rel(m0, ref.mean(0)) < 1e-5
    assert rel(i1, i0) < 1e-6


# (n, cin, h, w, cout, k, stride, pad, dil, bias): a split-K grid (few tiles), a large unsplit
# grid with bias (VGG-like: the vector epilogue with biases), a ragged one (per-element path),
# and the stride-2 parity data gradient
EPI_SHAPES = [(1, 64, 9, 11, 64, 3, 1, 1, 1, True), (2, 128, 48, 64, 128, 3, 1, 1, 1, True),
              (1, 32, 13, 17, 36, 1, 1, 0, 1, False), (2, 64, 20, 24, 128, 1, 2, 0, 1, False)]


@pytest.mark.parametrize("shape", EPI_SHAPES, ids=[f"e{i}" for i in range(len(EPI_SHAPES))])
def test_epilogue_term_images_equal_the_split_of_the_output(shape):
    """Under F32X3 the _x forms' y_bf16 / dx_bf16 are the output's term images: the F32X3
    kernels' epilogues (and split-K reduce) now write them in the same pass as the fp32 output
    (conv_kernels.hpp epi_outb / epi_store_f32x4) instead of out_copy's pass over the finished
    output.  Either way they must be torch's exact three-term RNE split of the fp32 output,
    bitwise: forward with bias + ReLU (DeeplabVGG's conv, deeplab_vgg.py:34-43), forward with the
    fused BN statistics, data gradient with the ReLU' epilogue on aux and with a residual."""
    k = K()
    n, cin, h, w, cout, ks, st, pd, dl, bias = shape
    g = torch.Generator().manual_seed(77)
    x = torch.randn(n, h, w, cin, generator=g).to(DEV)
    wt = (torch.randn(cout, ks, ks, cin, generator=g) * 0.1).to(DEV)
    b = torch.randn(cout, generator=g).to(DEV) if bias else None
    geo = k.ConvGeom(cin, cout, ks, ks, st, (pd,), (dl,))
    oh, ow = geo.out_hw(h, w)
    y, yt = k.conv_fwd(geo, x, n, h, w, [wt], [b] if bias else None, flags=k.EPI_RELU, bf16_out=True)
    assert yt.shape == (n, oh, ow, 3, cout)
    assert torch.equal(yt, terms(y)), "forward bias + ReLU"
    if not bias:
        y2, _st = k.conv_fwd_bnstats(geo, x, n, h, w, [wt])
        y3 = k.conv_fwd(geo, x, n, h, w, [wt])
        assert torch.equal(y2, y3)
    dy = torch.randn(n, oh, ow, cout, generator=g).to(DEV)
    aux = F.relu(torch.randn(n, h, w, cin, generator=g)).to(DEV)
    dx, dxt = k.conv_dgrad(geo, dy, n, h, w, [wt], aux=aux, flags=k.EPI_RELU_GRAD, bf16_out=True)
    assert torch.equal(dxt, terms(dx)), "data gradient with ReLU'"
    res = torch.randn(n, h, w, cin, generator=g).to(DEV)
    dx2, dxt2 = k.conv_dgrad(geo, dy, n, h, w, [wt], res=res, bf16_out=True)
    assert torch.equal(dxt2, terms(dx2)), "data gradient with residual"
