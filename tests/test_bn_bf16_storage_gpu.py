"""BatchNorm passes on bf16 activation storage (config c5, bf16 conv maths): x, the residual and
the saved output y stored bf16, gradients fp32.

The passes give each thread two channel quads (one 16-B load of eight bf16) when C % 8 == 0 and
every operand is 16-B aligned, else one quad (8-B loads, the fp32 passes' layout).  Both layouts
are checked against an fp64 restatement of the same BN on the same bf16 values, and against
each other (a misaligned view forces one quad).  Reference: model/deeplab_multi.py:65-101
(Bottleneck BN + ReLU + residual) under torch.autocast(bfloat16) storage.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def K():
    from adaptsegnet_amd import kernels
    prev = kernels.get_conv_math()
    kernels.set_conv_math(kernels.MATH_BF16)   # bf16 activation storage is the bf16 maths'
    yield kernels
    kernels.set_conv_math(prev)


def misaligned(t):
    """The same values in storage offset by 8 B (16-B loads impossible: one quad a thread)."""
    off = 8 // t.element_size()
    buf = torch.empty(t.numel() + off, dtype=t.dtype, device=t.device)
    v = buf[off:].view(t.shape)
    v.copy_(t)
    assert v.data_ptr() % 16 == 8
    return v


def close_bf16(a, ref):
    """a (bf16) is ref rounded to bf16 up to the fp32 arithmetic before the rounding: within
    one bf16 ulp (2^-8 relative) of each value plus 1e-4 of the tensor's scale (the fp32
    statistics' relative error times |x - mean|, which dominates where the residual add or the
    affine cancels to small outputs)."""
    a, ref = a.double(), ref.double()
    tol = 2.0 ** -8 * ref.abs() + 1e-4 * float(ref.abs().max())
    return bool(((a - ref).abs() <= tol).all())


def ref_forward(x, res, w, b, relu):
    xd = x.double()
    mean = xd.mean(0)
    var = xd.var(0, unbiased=False)
    invstd = 1.0 / torch.sqrt(var + 1e-5)
    y = (xd - mean) * invstd * w.double() + b.double()
    if res is not None:
        y = y + res.double()
    return (y.clamp_min(0) if relu else y), mean, invstd


@pytest.mark.parametrize("rows,c,with_res", [(4 * 37 * 53, 256, True), (3 * 41 * 29 + 7, 64, False),
                                             (2 * 33 * 17, 1024, True), (1999, 12, False)])
def test_bn_forward_on_bf16_storage(K, rows, c, with_res):
    g = torch.Generator().manual_seed(rows + c)
    x = (torch.randn(rows, c, generator=g) * 2 + 0.5).to(DEV).to(torch.bfloat16)
    res = torch.randn(rows, c, generator=g).to(DEV).to(torch.bfloat16) if with_res else None
    w, b = torch.rand(c, generator=g).to(DEV) + 0.5, torch.randn(c, generator=g).to(DEV) * 0.1
    outs = []
    for xx, rr in ((x, res), (misaligned(x), misaligned(res) if res is not None else None)):
        rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
        _, mean, invstd, yb = K.bn_fwd_train(xx, w, b, rm, rv, 0.1, 1e-5, res=rr, relu=True, bf16_out=True,
                                             fp32_out=False)
        outs.append((yb, mean, invstd, rm, rv))
    yref, mref, iref = ref_forward(x, res, w, b, True)
    for yb, mean, invstd, rm, rv in outs:
        assert yb.dtype == torch.bfloat16 and yb.shape == (rows, c)
        assert float((mean.double() - mref).abs().max()) < 1e-5 * (1 + float(mref.abs().max()))
        assert float(((invstd.double() - iref) / iref).abs().max()) < 1e-5
        assert torch.allclose(rm.double(), 0.1 * mref, rtol=1e-5, atol=1e-6)
        assert close_bf16(yb, yref)
    # the two layouts: the same statistics up to fp32 summation order
    assert close_bf16(outs[0][0], outs[1][0].double())
    assert float(((outs[0][2] - outs[1][2]) / outs[1][2]).abs().max()) < 1e-6


@pytest.mark.parametrize("rows,c,mask_from_y", [(4 * 37 * 53, 256, True), (3 * 41 * 29 + 7, 64, False),
                                                (2 * 33 * 17, 1024, True), (1999, 12, False)])
def test_bn_backward_on_bf16_storage(K, rows, c, mask_from_y):
    g = torch.Generator().manual_seed(7 * rows + c)
    x = (torch.randn(rows, c, generator=g) * 2 + 0.5).to(DEV).to(torch.bfloat16)
    res = torch.randn(rows, c, generator=g).to(DEV).to(torch.bfloat16) if mask_from_y else None
    w, b = torch.rand(c, generator=g).to(DEV) + 0.5, torch.randn(c, generator=g).to(DEV) * 0.1
    _, mean, invstd, yb = K.bn_fwd_train(x, w, b, None, None, 0.1, 1e-5, res=res, relu=True, bf16_out=True,
                                         fp32_out=False)
    dy = torch.randn(rows, c, generator=g).to(DEV)
    # reference on the same bf16 values and the kernel's own statistics
    xd, md, idd = x.double(), mean.double(), invstd.double()
    xhat = (xd - md) * idd
    o = yb.double() if mask_from_y else xhat * w.double() + b.double()
    gg = dy.double() * (o > 0)
    dref = w.double() * idd * (gg - gg.mean(0) - xhat * (gg * xhat).mean(0))
    outs = []
    for dd, yy, xx in ((dy, yb, x), (misaligned(dy), misaligned(yb), misaligned(x))):
        dres = torch.empty(rows, c, device=DEV) if mask_from_y else None
        _, dxb = K.bn_bwd(dd, yy if mask_from_y else None, xx, w, mean, invstd, relu=True, dres=dres, bias=b,
                          bf16_out=True, fp32_out=False)
        outs.append((dxb, dres))
        if mask_from_y:
            assert torch.equal(dres, dy * (yb.float() > 0))
        scale = float(dref.abs().max())
        assert float((dxb.double() - dref).abs().max()) < 2 ** -8 * scale + 1e-6, (rows, c)
    assert float((outs[0][0].double() - outs[1][0].double()).abs().max()) <= 2 ** -7 * float(dref.abs().max())
