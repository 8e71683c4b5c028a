"""Host-side planning of the operand copies (no GPU): which fp32 activations the bf16 program
skips writing, and the host checks of the _x entry points.

engine.bf16_only() lets a BatchNorm pass write ONLY the bf16 copy of its output when every
consumer product runs on a kernel that reads only that copy.  The decision comes from the
library's own plan (adaptseg_conv2d_copy_operand_only), the same plan the _x entry points check
a NULL fp32 operand against.
"""
import ctypes

import pytest

from adaptsegnet_amd import _lib


def _bf16(K):
    K.set_conv_math(K.MATH_BF16)


def _block_decisions(model, n, h, w):
    """The engine's bf16_only() calls of one DeeplabMulti forward + backward in train mode
    (engine.block_forward / block_backward), in program order: [(site, decision)]."""
    from adaptsegnet_amd import engine
    out = []
    gs = model.conv1.geom()
    h, w = gs.out_hw(h, w)
    h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1   # maxpool 3x3/2 p1
    first = True   # the stem's maxpool output has no bf16 copy (xb is None for the first block)
    for li, layer in enumerate((model.layer1, model.layer2, model.layer3, model.layer4), 1):
        for bi, blk in enumerate(layer):
            g1, g2, g3 = blk.conv1.geom(), blk.conv2.geom(), blk.conv3.geom()
            oh, ow = g1.out_hw(h, w)
            name = f"layer{li}.{bi}"
            out.append((f"{name}.y1", engine.bf16_only(g2, n, oh, ow, (0, 2))))
            out.append((f"{name}.y2", engine.bf16_only(g3, n, oh, ow, (0, 2))))
            out.append((f"{name}.dc3", engine.bf16_only(g3, n, oh, ow, (1, 2))))
            out.append((f"{name}.dy2", engine.bf16_only(g2, n, oh, ow, (1, 2))))
            if not first:
                out.append((f"{name}.dy1", engine.bf16_only(g1, n, h, w, (1, 2))))
                if blk.downsample is not None:
                    out.append((f"{name}.gd", engine.bf16_only(blk.downsample[0].geom(), n, h, w, (1, 2))))
            first = False
            h, w = oh, ow
    return out


def test_skip_decisions_match_across_geometries_but_the_kernel_variants_do_not():
    """What the full-geometry c5 test (test_fullres_gpu.py::test_fullres_c5_bf16_*) adds over the
    41x57 model tests.  The skip decisions depend on the channel counts only (N >= 128, Cin %
    8), so 41x57 and 1280x720 / 1024x512 skip the SAME fp32 tensors (measured: 158 of 167
    sites); the kernel variants that read the copies differ (K split or not, K step 32 / 64),
    and those are what the full geometry exercises."""
    import bench
    from adaptsegnet_amd import kernels as K
    from adaptsegnet_amd.model import DeeplabMulti, FCDiscriminator
    model, D = DeeplabMulti(num_classes=19), FCDiscriminator(num_classes=19)
    prev = K.get_conv_math()
    _bf16(K)
    try:
        small = _block_decisions(model, 2, 41, 57) + _block_decisions(model, 2, 33, 49)
        full = _block_decisions(model, 1, 720, 1280) + _block_decisions(model, 1, 512, 1024)
        p_small, p_full = set(), set()
        bench.conv_inventory(model, D, "multi-level", 2, (57, 41), (49, 33), (49, 33), products=p_small)
        bench.conv_inventory(model, D, "multi-level", 1, (1280, 720), (1024, 512), (1024, 512), products=p_full)
    finally:
        K.set_conv_math(prev)
    assert [s for s, _ in small] == [s for s, _ in full]
    assert [v for _, v in small] == [v for _, v in full]
    assert sum(v for _, v in full) > len(full) // 2
    only_full = sorted(p_full - p_small)
    print(f"(op, selector, split-K) launched only at the full geometry: {only_full}")
    assert only_full, "the full geometry would run no kernel variant the 41x57 tests do not"


def test_copy_operand_only_matches_the_lds_dma_selectors():
    """adaptseg_conv2d_copy_operand_only (what engine.bf16_only asks) is exactly the set of
    products the planner puts on the LDS-DMA kernels (selectors 100*op + 94 / 97-99, 192 / 193)
    or the register-staged bf16 forward (90-93), for every conv geometry of the c5 step; under
    F32X3 it is exactly the set the term-image kernel takes when the copies are passed
    (selectors 100*op + 88 / 89, conv_x3r.hpp); under the fp32-input MFMA math never."""
    import bench
    from adaptsegnet_amd import kernels as K
    from adaptsegnet_amd.model import DeeplabMulti, FCDiscriminator
    model, D = DeeplabMulti(num_classes=19), FCDiscriminator(num_classes=19)
    geoms = []
    orig = K.conv_kernel_id

    def spy(g, n, h, w, op, strides=None, copies=False):
        geoms.append((g, n, h, w, op, strides))
        return orig(g, n, h, w, op, strides, copies=copies)

    prev = K.get_conv_math()
    K.conv_kernel_id = spy
    try:
        _bf16(K)
        bench.conv_inventory(model, D, "multi-level", 4, (1280, 720), (1024, 512), (1024, 512))
        bench.conv_inventory(model, D, "multi-level", 2, (57, 41), (49, 33), (49, 33))
    finally:
        K.conv_kernel_id = orig
    try:
        seen = set()
        for g, n, h, w, op, st in geoms:
            kid, _ = K.conv_kernel_id(g, n, h, w, op, st)
            lds_dma = kid % 100 in (85, 94, 97, 98, 99) or (op == 1 and kid % 100 in (92, 93))
            # the register-staged bf16 forward (90-93) reads the contiguous bf16 copy too
            lds_dma = lds_dma or (op == 0 and kid % 100 in (90, 91, 92, 93))
            if g.cout <= 32:   # tap-GEMM (ASPP heads): the selector is the inner GEMM's, whose
                # forward / weight gradient read x's copy; its data gradient's tap scatter and
                # the thin (Cout 1) discriminator head read fp32
                lds_dma = lds_dma and op != 1 and len(g.pads) > 1
            assert K.conv_copy_operand_only(g, n, h, w, op, st) == lds_dma, (g, n, h, w, op, kid)
            seen.add(lds_dma)
        assert seen == {True, False}
        K.set_conv_math(K.MATH_F32X3)
        seen = set()
        for g, n, h, w, op, st in geoms:
            kid, _ = K.conv_kernel_id(g, n, h, w, op, st, copies=True)
            x3r = kid % 100 in (88, 89)
            assert K.conv_copy_operand_only(g, n, h, w, op, st) == x3r, (g, n, h, w, op, kid)
            seen.add(x3r)
        assert seen == {True, False}
        K.set_conv_math(K.MATH_F32)
        for g, n, h, w, op, st in geoms[:200]:
            assert not K.conv_copy_operand_only(g, n, h, w, op, st)
    finally:
        K.set_conv_math(prev)


@pytest.mark.parametrize("op", [0, 1, 2])
def test_null_fp32_operand_with_misaligned_weight_is_rejected_on_host(op):
    """a misaligned weight (or operand) clears the LDS-DMA plan at launch time; a NULL
    fp32 operand must then be rejected with ADAPTSEG_ERR_ARG before any launch, not handed to
    the fp32 kernel."""
    from adaptsegnet_amd import kernels as K
    L = _lib.lib()
    prev = K.get_conv_math()
    _bf16(K)
    try:
        g = K.ConvGeom(256, 256, 3, 3, 1, (2,), (2,))
        d = K._desc(g, 4, 64, 128, K.nhwc_strides(4, 64, 128, 256))[0]
        assert K.conv_copy_operand_only(g, 4, 64, 128, op)
        aligned, misaligned = ctypes.c_void_p(4096), _lib.ptr_array([4096 + 4])
        if op == 0:
            st = L.adaptseg_conv2d_fwd_x(ctypes.byref(d), None, aligned, misaligned, None, None, None,
                                         ctypes.c_void_p(8192), None, 0, None, 0, None)
            assert st == 1 and b"fp32 input" in L.adaptseg_last_error()
            nt = ctypes.c_int(0)
            st = L.adaptseg_conv2d_fwd_bnstats_x(ctypes.byref(d), None, aligned, misaligned, None, ctypes.c_void_p(8192), None,
                                                 ctypes.c_void_p(16384), 1 << 20, ctypes.byref(nt), None, 0, None)
            assert st == 1 and b"fp32 input" in L.adaptseg_last_error()
        elif op == 1:
            st = L.adaptseg_conv2d_bwd_data_x(ctypes.byref(d), None, aligned, misaligned, None, None, None,
                                              ctypes.c_void_p(8192), None, 0, None, 0, None)
            assert st == 1 and b"fp32 dY" in L.adaptseg_last_error()
        else:   # weight gradient: fp32 x present but misaligned, dY only as a copy
            st = L.adaptseg_conv2d_bwd_weight_x(ctypes.byref(d), None, aligned, ctypes.c_void_p(4096 + 4), aligned,
                                                _lib.ptr_array([8192]), None, 0, None, 0, None)
            assert st == 1 and b"fp32 operands" in L.adaptseg_last_error()
    finally:
        K.set_conv_math(prev)


def test_weight_pack_sizes_follow_the_plan():
    """adaptseg_conv2d_wpack_size: the F32X3 forward / data-gradient products read a three-term
    pack (6 B per weight, rows padded to 128-wide tiles), the bf16 ones a bf16 pack (2 B), the
    weight gradients, thin (Cout <= 4) and tap-GEMM (ASPP) products none."""
    from adaptsegnet_amd import kernels as K

    def size(g, op, n=2, h=32, w=48):
        d = K._desc(g, n, h, w, K.nhwc_strides(n, h, w, g.cin))[0]
        b = ctypes.c_size_t(0)
        assert _lib.lib().adaptseg_conv2d_wpack_size(ctypes.byref(d), op, ctypes.byref(b)) == 0
        return b.value

    g = K.ConvGeom(256, 512, 3, 3, 1, (2,), (2,))
    assert size(g, 0) == 3 * 512 * 9 * 256 * 2 and size(g, 1) == 3 * 256 * 9 * 512 * 2 and size(g, 2) == 0
    assert size(K.ConvGeom(512, 1, 4, 4, 2, (1,), (1,)), 0) == 0                          # thin
    assert size(K.ConvGeom(2048, 19, 3, 3, 1, (6, 12, 18, 24), (6, 12, 18, 24)), 0) == 0  # tap-GEMM
    prev = K.get_conv_math()
    try:
        K.set_conv_math(K.MATH_BF16)
        assert size(g, 0) == 512 * 9 * 256 * 2 and size(g, 1) == 256 * 9 * 512 * 2
        K.set_conv_math(K.MATH_F32)
        assert size(g, 0) == 0
    finally:
        K.set_conv_math(prev)


def test_f32x3_forward_term_images_only_for_the_wide_dilated_convs(monkeypatch):
    """Under the default F32X3 maths the engine writes no operand copies (X3_FWD_TERMS 0 since
    round 6: layers 3-4 conv2 run on the x3h tile over fp32 operands, selector 86).  With
    X3_FWD_TERMS 1 it writes one: y1's three bf16 terms, for the forward of conv2 in layers 3-4
    (dilated 3x3, Cin >= 256), which then runs on the term-image kernel (selector 88,
    conv_x3r.hpp); every other product keeps the fp32 kernels.  bench.conv_inventory books
    those FLOPs under the selector that runs."""
    import bench
    from adaptsegnet_amd import engine
    from adaptsegnet_amd import kernels as K
    from adaptsegnet_amd.model import DeeplabMulti, FCDiscriminator
    assert K.get_conv_math() == K.MATH_F32X3 and not engine.bf16_operands()
    model, D = DeeplabMulti(num_classes=19), FCDiscriminator(num_classes=19)
    convs2 = [b.conv2.geom() for b in list(model.layer3) + list(model.layer4)]
    n, h, w = 4, 64, 128   # layers 3-4 at 1024x512 (stem /2, max-pool /2 floor, layer2 /2)
    flops = 2 * sum(g.flops(n, h, w) for g in convs2)   # source + target forwards
    assert engine.X3_FWD_TERMS == 0
    assert not any(engine.x3_forward_terms(blk.conv2.geom()) for layer in (model.layer1, model.layer2,
                   model.layer3, model.layer4) for blk in layer)
    inv = bench.conv_inventory(model, D, "single-level", 4, (1024, 512), (1024, 512), (1024, 512))
    assert inv.get(88, 0.0) == 0.0 and inv[86] >= flops
    monkeypatch.setattr(engine, "X3_FWD_TERMS", 1)
    want = set()
    for li, layer in enumerate((model.layer1, model.layer2, model.layer3, model.layer4), 1):
        for blk in layer:
            for conv in (blk.conv1, blk.conv2, blk.conv3):
                on = engine.x3_forward_terms(conv.geom())
                assert on == (conv is blk.conv2 and li >= 3), (li, conv)
                if on:
                    want.add(conv.geom())
    inv = bench.conv_inventory(model, D, "single-level", 4, (1024, 512), (1024, 512), (1024, 512))
    assert abs(inv[88] - flops) <= 1e-6 * flops
    K.set_conv_math(K.MATH_F32)
    try:
        assert not any(engine.x3_forward_terms(g) for g in want)
    finally:
        K.set_conv_math(K.MATH_F32X3)


def test_inventory_counts_only_the_forwards_that_run():
    """bench.conv_inventory books the discriminator forward the D step reuses (StepConfig.d_reuse)
    and the single-level step's discarded first head (second_head_only) only when they run."""
    import bench
    from adaptsegnet_amd import engine
    from adaptsegnet_amd.model import DeeplabMulti, FCDiscriminator
    model, D = DeeplabMulti(num_classes=19), FCDiscriminator(num_classes=19)
    args = (model, D, "single-level", 4, (1024, 512), (1024, 512), (1024, 512))
    base = sum(bench.conv_inventory(*args).values())
    n, h, w = 4, 512, 1024
    d_fwd = 0.0
    for conv in D._convs():
        g = conv.geom()
        d_fwd += g.flops(n, h, w)
        h, w = g.out_hw(h, w)
    assert abs(sum(bench.conv_inventory(*args, d_reuse=False).values()) - base - d_fwd) <= 1e-9 * base
    head = engine.aspp_geom(model.layer5).flops(4, 64, 128) * 2   # layer5 at 1024x512 (64 x 128), source + target
    assert abs(sum(bench.conv_inventory(*args, first_head=True).values()) - base - head) <= 1e-9 * base
    multi = (model, D, "multi-level", 2, (1280, 720), (1024, 512), (1024, 512))
    assert bench.conv_inventory(*multi, first_head=True) == bench.conv_inventory(*multi)
