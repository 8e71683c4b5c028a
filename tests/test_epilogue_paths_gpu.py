"""The conv epilogue's two store paths give the same bits (conv_kernels.hpp igemm_epilogue).

Full tiles of the F32X3 and bf16 LDS-DMA kernels store through a per-wave LDS transpose with
16-B rows (epi_store_f32x4 / epi_store_bf16x8); any tile whose output is not 16-B aligned takes
the per-element path.  Same kernel, same accumulation, same epilogue arithmetic order — so an
output placed at a 16-B-aligned address and the same output one element off it must be
bitwise equal, for the plain store, the in-place residual (with its ReLU-mask bitmap), the
accumulate and the stride-2 LeakyReLU-gradient data gradient (parity-class scatter), under both
conv maths.  Reference: the Bottleneck's data gradient with its
residual, model/deeplab_multi.py:96-103.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def K():
    from adaptsegnet_amd import kernels
    return kernels


def off_by_one(t):
    """A copy of t one element past a 16-B boundary (the per-element epilogue path)."""
    buf = torch.empty(t.numel() + 8, dtype=t.dtype, device=t.device)
    v = buf[1:1 + t.numel()].view(t.shape)
    assert v.data_ptr() % 16 != 0
    v.copy_(t)
    return v


def terms(t):
    hi = t.to(torch.bfloat16)
    r1 = t - hi.float()
    mid = r1.to(torch.bfloat16)
    return torch.stack([hi, mid, (r1 - mid.float()).to(torch.bfloat16)], dim=-2)


CASES = ["f32x3_fwd", "f32x3_dgrad_res_bits", "f32x3_dgrad_acc", "f32x3_x3r_dgrad", "f32x3_s2_leaky_grad",
         "bf16_dgrad_res", "bf16_dgrad_acc"]


@pytest.mark.parametrize("case", CASES)
def test_vector_and_per_element_epilogues_agree_bitwise(case):
    k = K()
    prev = k.get_conv_math()
    bf16 = case.startswith("bf16")
    k.set_conv_math(k.MATH_BF16 if bf16 else k.MATH_F32X3)
    try:
        g = torch.Generator().manual_seed(len(case))
        n, h, w = 2, 32, 64            # 4096 rows: whole 128- / 256-row tiles
        cin, cout, ks, dil = (256, 256, 3, 2) if "x3r" in case else (256, 512, 1, 1)
        geom = k.ConvGeom(cin, cout, ks, ks, 1, (dil * (ks // 2),), (dil,))
        if "s2" in case:   # the discriminator's 4x4 / 2 conv: data gradient by parity class, LeakyReLU'
            n, h, w, cin, cout, ks = 2, 64, 128, 128, 256, 4
            geom = k.ConvGeom(cin, cout, ks, ks, 2, (1,), (1,))
        oh, ow = geom.out_hw(h, w)
        wt = [(torch.randn(cout, ks, ks, cin, generator=g) / (cin * ks * ks) ** 0.5).to(DEV)]
        if case == "f32x3_fwd":
            x = torch.randn(n, h, w, cin, generator=g).to(DEV)
            a = torch.empty(n, h, w, cout, device=DEV)
            b = off_by_one(a)
            k.conv_fwd(geom, x, n, h, w, wt, out=a)
            k.conv_fwd(geom, x, n, h, w, wt, out=b)
        else:
            dy = torch.randn(n, oh, ow, cout, generator=g).to(DEV)
            dyb = dy.to(torch.bfloat16) if bf16 else (terms(dy) if "x3r" in case else None)
            base = torch.randn(n, h, w, cin, generator=g).to(DEV)
            if bf16:
                base = base.to(torch.bfloat16)
            a, b = base.clone(), off_by_one(base)
            if case.endswith("acc"):
                for o in (a, b):
                    k.conv_dgrad(geom, None if bf16 else dy, n, h, w, wt, out=o, flags=k.EPI_ACCUMULATE, dyb=dyb)
            elif "res" in case:
                bits = None
                if case.endswith("bits"):
                    bits = k.mask_bits_like(base)
                    bits.copy_(torch.randint(-2 ** 31, 2 ** 31 - 1, bits.shape, generator=g,
                                             dtype=torch.int64).to(torch.int32))
                if bf16:   # a bf16 residual must be 16-B aligned (adaptseg_conv2d_bwd_data_xg): not in place
                    for o in (a, b):
                        k.conv_dgrad(geom, None, n, h, w, wt, out=o, res=base, dyb=dyb)
                else:
                    for o in (a, b):   # the in-place residual: dx = dgrad + g over g
                        k.conv_dgrad(geom, dy, n, h, w, wt, out=o, res=o, dyb=dyb, resbits=bits)
            elif "leaky" in case:
                aux = torch.randn(n, h, w, cin, generator=g).to(DEV)   # the activation output (its sign)
                for o in (a, b):
                    k.conv_dgrad(geom, dy, n, h, w, wt, out=o, aux=aux)
            else:
                for o in (a, b):
                    k.conv_dgrad(geom, dy, n, h, w, wt, out=o, dyb=dyb)
        torch.cuda.synchronize()
        assert torch.equal(a, b), (a.float() - b.float()).abs().max().item()
        assert torch.isfinite(a.float()).all()
    finally:
        k.set_conv_math(prev)
