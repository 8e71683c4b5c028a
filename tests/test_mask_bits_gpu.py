"""ReLU mask bitmaps of the Bottleneck's output (engine.MASK_BITS): BN3's forward apply writes
bit (y > 0) per element beside y, and the backward reads those bits instead of the stored block
output — BN3's backward (g = gout * bit, adaptseg_bn_bwd_xg dy_bits), the downsample BN's
backward (same g) and the identity residual in conv1's data-gradient epilogue
(adaptseg_conv2d_bwd_data_xg res_bits).  Reference: model/deeplab_multi.py:96-103
(out += residual; out = relu(out)).

Checked bitwise: the bits equal (y > 0) from every forward apply variant (fp32, bf16 storage
with one and two channel quads a thread, term-image residual, eval mode); a backward reading
the bits equals the backward on the explicitly masked gradient; a masked-residual data gradient
equals the data gradient on the explicitly masked residual.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def K():
    from adaptsegnet_amd import kernels
    return kernels


def unpack(bits, c):
    """int32 [rows, c/32] -> bool [rows, c]"""
    b = bits.to(torch.int64) & 0xFFFFFFFF
    sh = torch.arange(32, device=bits.device)
    return ((b.unsqueeze(-1) >> sh) & 1).bool().reshape(bits.shape[0], c)


def misaligned(t):
    off = 8 // t.element_size()
    buf = torch.empty(t.numel() + off, dtype=t.dtype, device=t.device)
    v = buf[off:].view(t.shape)
    v.copy_(t)
    return v


@pytest.mark.parametrize("storage", ["f32", "bf16", "bf16_misaligned", "f32_terms_res"])
@pytest.mark.parametrize("rows,c", [(3 * 37 * 41, 256), (2 * 29 * 31 + 5, 1024), (777, 32)])
def test_bn_forward_writes_the_relu_bits(storage, rows, c):
    k = K()
    prev = k.get_conv_math()
    k.set_conv_math(k.MATH_BF16 if storage.startswith("bf16") else k.MATH_F32X3)
    try:
        g = torch.Generator().manual_seed(rows + c)
        x = (torch.randn(rows, c, generator=g) * 2).to(DEV)
        res = torch.randn(rows, c, generator=g).to(DEV)
        w, b = torch.rand(c, generator=g).to(DEV) + 0.5, torch.randn(c, generator=g).to(DEV) * 0.3
        if storage.startswith("bf16"):
            x, res = x.to(torch.bfloat16), res.to(torch.bfloat16)
            if storage == "bf16_misaligned":
                x, res = misaligned(x), misaligned(res)
        if storage == "f32_terms_res":
            hi = res.to(torch.bfloat16)
            r1 = res - hi.float()
            mid = r1.to(torch.bfloat16)
            res = torch.stack([hi, mid, (r1 - mid.float()).to(torch.bfloat16)], dim=-2)
        bits = k.mask_bits_like(x)
        bf16 = storage.startswith("bf16")
        out = k.bn_fwd_train(x, w, b, None, None, 0.1, 1e-5, res=res, relu=True, bf16_out=bf16, fp32_out=not bf16,
                             ybits=bits)
        y = out[3] if bf16 else out[0]
        assert torch.equal(unpack(bits, c), (y.float() > 0).reshape(rows, c))
        # eval mode
        bits_e = k.mask_bits_like(x)
        rm, rv = torch.randn(c, generator=g).to(DEV) * 0.1, torch.rand(c, generator=g).to(DEV) + 0.5
        ye = k.bn_fwd_infer(x, w, b, rm, rv, 1e-5, res=res, relu=True, bf16_out=bf16, fp32_out=not bf16,
                            ybits=bits_e)
        ye = ye[1] if bf16 else ye
        assert torch.equal(unpack(bits_e, c), (ye.float() > 0).reshape(rows, c))
    finally:
        k.set_conv_math(prev)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("train", [True, False])
def test_bn_backward_with_bits_equals_masked_gradient(dtype, train):
    k = K()
    prev = k.get_conv_math()
    k.set_conv_math(k.MATH_BF16 if dtype == torch.bfloat16 else k.MATH_F32X3)
    try:
        g = torch.Generator().manual_seed(17)
        rows, c = 2 * 33 * 37, 512
        x = (torch.randn(rows, c, generator=g) * 2).to(DEV).to(dtype)
        res = torch.randn(rows, c, generator=g).to(DEV).to(dtype)
        w, b = torch.rand(c, generator=g).to(DEV) + 0.5, torch.randn(c, generator=g).to(DEV) * 0.3
        bits = k.mask_bits_like(x)
        bf16 = dtype == torch.bfloat16
        out = k.bn_fwd_train(x, w, b, None, None, 0.1, 1e-5, res=res, relu=True, bf16_out=bf16, fp32_out=not bf16,
                             ybits=bits)
        mean, invstd = out[1], out[2]
        if not train:
            mean, invstd = torch.randn(c, generator=g).to(DEV) * 0.1, torch.rand(c, generator=g).to(DEV) + 0.5
        dy = torch.randn(rows, c, generator=g).to(DEV).to(dtype)   # bf16 dy: bf16 gradient storage
        m = unpack(bits, c)
        dym = torch.where(m, dy, torch.zeros_like(dy))
        a = k.bn_bwd(dy, None, x, w, mean, invstd, relu=False, train=train, bias=b, bf16_out=True, fp32_out=not bf16,
                     dybits=bits)
        ref = k.bn_bwd(dym, None, x, w, mean, invstd, relu=False, train=train, bias=b, bf16_out=True,
                       fp32_out=not bf16)
        assert torch.equal(a[1], ref[1])
        if not bf16:
            assert torch.equal(a[0], ref[0])
    finally:
        k.set_conv_math(prev)


@pytest.mark.parametrize("math", ["f32x3", "bf16"])
def test_conv_dgrad_masked_residual_equals_masked_input(math):
    k = K()
    prev = k.get_conv_math()
    k.set_conv_math(k.MATH_BF16 if math == "bf16" else k.MATH_F32X3)
    try:
        g = torch.Generator().manual_seed(23)
        for n, cin, h, w, cout in ((2, 1024, 16, 24, 256), (2, 256, 40, 48, 64)):
            geom = k.ConvGeom(cin, cout, 1, 1, 1, (0,), (1,))
            wd = [(torch.randn(cout, 1, 1, cin, generator=g) / cin ** 0.5).to(DEV)]
            dy = torch.randn(n, h, w, cout, generator=g).to(DEV)
            dyb = dy.to(torch.bfloat16) if math == "bf16" else None
            res = torch.randn(n, h, w, cin, generator=g).to(DEV)
            bits = k.mask_bits_like(res)
            bits.copy_(torch.randint(-2 ** 31, 2 ** 31 - 1, bits.shape, generator=g, dtype=torch.int64).to(torch.int32))
            m = unpack(bits, cin).reshape(n, h, w, cin)
            resm = torch.where(m, res, torch.zeros_like(res))
            a = k.conv_dgrad(geom, dy, n, h, w, wd, res=res.clone(), resbits=bits, dyb=dyb)
            ref = k.conv_dgrad(geom, dy, n, h, w, wd, res=resm, dyb=dyb)
            assert torch.equal(a, ref)
            if math == "bf16":   # bf16 gradient storage: bf16 residual, bf16-only output, in place
                rb = res.to(torch.bfloat16)
                rbm = torch.where(m, rb, torch.zeros_like(rb))
                a = k.conv_dgrad(geom, None, n, h, w, wd, out=rb.clone(), res=None, dyb=dyb)   # warm (no residual)
                a = rb.clone()
                k.conv_dgrad(geom, None, n, h, w, wd, out=a, res=a, resbits=bits, dyb=dyb)
                ref = k.conv_dgrad(geom, None, n, h, w, wd, res=rbm, dyb=dyb, bf16_only=True)
                assert torch.equal(a, ref)
    finally:
        k.set_conv_math(prev)
