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


@pytest.mark.parametrize("rows,c,mask_from_y,train", [(4 * 37 * 53, 256, True, True), (3 * 41 * 29 + 7, 64, False, True),
                                                      (2 * 33 * 17, 1024, True, True), (1999, 12, False, True),
                                                      (2 * 33 * 17, 1024, True, False)])
def test_bn_backward_on_bf16_gradient_storage(K, rows, c, mask_from_y, train):
    """bf16 GRADIENT storage (engine.lowp_grads, adaptseg_bn_bwd_xg): dy is a bf16 tensor, the
    residual gradient dres is written over it in bf16 (in place, as block_backward does with the
    residual stream), dx as its bf16 copy only.  Against the fp64 restatement on the same bf16
    values: dres exactly dy*mask (masking is exact in bf16), dx within one bf16 ulp of the scale;
    both thread layouts (the 16-B one and, misaligned, one quad a thread); eval mode too."""
    g = torch.Generator().manual_seed(11 * rows + c)
    x = (torch.randn(rows, c, generator=g) * 2 + 0.5).to(DEV).to(torch.bfloat16)
    res = torch.randn(rows, c, generator=g).to(DEV).to(torch.bfloat16) if mask_from_y else None
    w, b = torch.rand(c, generator=g).to(DEV) + 0.5, torch.randn(c, generator=g).to(DEV) * 0.1
    rm, rv = torch.randn(c, generator=g).to(DEV) * 0.1, torch.rand(c, generator=g).to(DEV) + 0.5
    _, mean, invstd, yb = K.bn_fwd_train(x, w, b, None, None, 0.1, 1e-5, res=res, relu=True, bf16_out=True,
                                         fp32_out=False)
    if not train:
        mean, invstd = rm, torch.rsqrt(rv + 1e-5)
    dy = torch.randn(rows, c, generator=g).to(DEV).to(torch.bfloat16)
    xd, md, idd = x.double(), mean.double(), invstd.double()
    xhat = (xd - md) * idd
    o = yb.double() if mask_from_y else xhat * w.double() + b.double()
    gg = dy.double() * (o > 0)
    if train:
        dref = w.double() * idd * (gg - gg.mean(0) - xhat * (gg * xhat).mean(0))
    else:
        dref = gg * w.double() * idd
    scale = float(dref.abs().max())
    for aligned in (True, False):
        dd = dy.clone() if aligned else misaligned(dy)
        yy, xx = (yb, x) if aligned else (misaligned(yb), misaligned(x))
        _, dxb = K.bn_bwd(dd, yy if (mask_from_y or not train) else None, xx, w, mean, invstd, relu=True,
                          dres=dd if mask_from_y else None, bias=b, bf16_out=True, fp32_out=False, train=train)
        assert dxb.dtype == torch.bfloat16
        if mask_from_y:
            assert dd.dtype == torch.bfloat16 and torch.equal(dd.double(), dy.double() * (o > 0))
        assert float((dxb.double() - dref).abs().max()) < 2 ** -8 * scale + 1e-6, (rows, c, aligned)


def test_conv_dgrad_bf16_gradient_storage(K):
    """bf16 gradient storage in the conv data gradient (adaptseg_conv2d_bwd_data_xg): the identity
    residual read in bf16 and the output stored bf16-only (block_backward's dx = dgrad(conv1) + g),
    fp32 residual into a bf16 output and bf16 residual into an fp32 output (the blocks whose input
    gradient changes storage), and EPI_ACCUMULATE into a bf16 output (the downsample block).
    Against fp64 on the same bf16 operands, the result rounded to bf16: within one bf16 ulp (RNE
    of an fp32 value that is itself within 1e-5 of the exact sum).  Shapes with and without split-K."""
    for n, cin, h, w, cout in ((2, 1024, 16, 24, 256), (2, 512, 64, 96, 128)):
        geom = K.ConvGeom(cin, cout, 1, 1, 1, (0,), (1,))
        g = torch.Generator().manual_seed(cin + h)
        wt = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
        dy = torch.randn(n, h, w, cout, generator=g)
        res = torch.randn(n, h, w, cin, generator=g)
        wb, dyb, resb = (t.to(torch.bfloat16).double() for t in (wt, dy, res))
        ref = torch.einsum("nhwo,oi->nhwi", dyb, wb[:, :, 0, 0])
        wd = [wt.permute(0, 2, 3, 1).contiguous().to(DEV)]
        dyd = dy.to(DEV).to(torch.bfloat16)
        tol = lambda r: 2.0 ** -8 * r.abs() + 1e-5 * float(r.abs().max())   # noqa: E731

        def ok(got, r):
            return bool(((got.double().cpu() - r).abs() <= tol(r)).all())

        # bf16 residual, bf16-only output, in place (the identity block)
        gb = res.to(DEV).to(torch.bfloat16)
        out = K.conv_dgrad(geom, None, n, h, w, wd, out=gb, res=gb, dyb=dyd)
        assert out is gb and out.dtype == torch.bfloat16 and ok(out, ref + resb)
        # fp32 residual -> bf16 output; bf16 residual -> fp32 output
        ob = K.conv_dgrad(geom, None, n, h, w, wd, res=res.to(DEV), dyb=dyd, bf16_only=True)
        assert ob.dtype == torch.bfloat16 and ok(ob, ref + res.double())
        of = torch.empty(n, h, w, cin, device=DEV)
        K.conv_dgrad(geom, None, n, h, w, wd, out=of, res=res.to(DEV).to(torch.bfloat16), dyb=dyd)
        assert float((of.double().cpu() - (ref + resb)).abs().max()) < 1e-5 * float((ref + resb).abs().max())
        # accumulate into a bf16 output
        acc = res.to(DEV).to(torch.bfloat16)
        K.conv_dgrad(geom, None, n, h, w, wd, out=acc, flags=K.EPI_ACCUMULATE, dyb=dyd)
        assert ok(acc, ref + resb)
