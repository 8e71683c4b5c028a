"""CPU: the C-ABI library loads (no GPU needed) and exports every symbol include/adaptseg.h declares."""
import ctypes
import os

import pytest

from adaptsegnet_amd import _lib


def test_library_exports_header_symbols():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) == set(_lib._SIGS), set(syms) ^ set(_lib._SIGS)


def test_version_and_error_paths_without_gpu():
    L = _lib.lib()
    assert b"gfx950" in L.adaptseg_version()
    # argument validation runs on the host: a bad descriptor is rejected before any launch
    d = _lib.ConvDesc()
    b = ctypes.c_size_t(0)
    assert L.adaptseg_conv2d_workspace_size(ctypes.byref(d), 0, ctypes.byref(b)) == 1
    assert b"bad" in L.adaptseg_last_error()


def test_default_conv_math_selects_f32x3():
    """The library's default conv math is F32X3: the vector products of the step run on the
    split-bf16 kernel (selector 100*op + 95, +1 for the stride-2 parity path); thin and
    per-element products keep their fp32 kernels.  F32X3_PRESPLIT moves the products whose
    operands come in 16-B chunks to the LDS-DMA kernels on pre-split images: 256x128x32 tiles
    (conv_x3r.hpp, 100*op + 88, + 89 for the stride-2 parity path / 128-row weight gradients)
    where a 32-deep step stays inside one tap (else the staged kernel);
    the stem's channel-padded weight gradient (Cin 4) stays on the staged one."""
    from adaptsegnet_amd import kernels as K
    assert K.get_conv_math() == K.MATH_F32X3
    g = K.ConvGeom(256, 256, 3, 3, 1, (2,), (2,))
    # the default ADAPTSEG_OPT_X3H 3: forward / data gradients with K >= 512 on the 256x128x32
    # tile splitting fp32 rows in-kernel (100*op + 86), weight gradients on the staged kernel
    assert K.get_x3h() == 3
    assert [K.conv_kernel_id(g, 4, 64, 128, op)[0] for op in (0, 1, 2)] == [86, 186, 295]
    c1 = K.ConvGeom(64, 256, 1, 1, 1, (0,), (1,))   # K 64: the staged kernel
    assert [K.conv_kernel_id(c1, 4, 128, 256, op)[0] for op in (0, 2)] == [95, 295]
    s2 = K.ConvGeom(256, 128, 1, 1, 2, (0,), (1,))
    assert K.conv_kernel_id(s2, 4, 128, 256, 1)[0] == 196   # stride-2 parity classes: staged
    K.set_x3h(0)
    try:
        assert [K.conv_kernel_id(g, 4, 64, 128, op)[0] for op in (0, 1, 2)] == [95, 195, 295]
    finally:
        K.set_x3h(3)
    stem = K.ConvGeom(3, 64, 7, 7, 2, (3,), (1,))
    assert K.conv_kernel_id(stem, 4, 512, 1024, 0, (3 * 512 * 1024, 512 * 1024, 1024, 1))[0] % 100 < 90
    d5 = K.ConvGeom(512, 1, 4, 4, 2, (1,), (1,))
    assert K.conv_kernel_id(d5, 4, 32, 64, 0)[0] == 80
    stem4 = K.ConvGeom(4, 64, 7, 7, 2, (3,), (1,))
    K.set_conv_math(K.MATH_F32X3_PRESPLIT)
    try:
        assert [K.conv_kernel_id(g, 4, 64, 128, op)[0] for op in (0, 1, 2)] == [88, 188, 288]
        assert K.conv_kernel_id(s2, 4, 128, 256, 1)[0] == 189
        g128 = K.ConvGeom(64, 128, 3, 3, 1, (1,), (1,))
        assert K.conv_kernel_id(g128, 4, 64, 128, 2)[0] == 289   # Cout < 256: 128-row tiles
        g16 = K.ConvGeom(48, 64, 3, 3, 1, (1,), (1,))
        assert [K.conv_kernel_id(g16, 4, 64, 128, op)[0] for op in (0, 1)] == [95, 188]
        assert K.conv_kernel_id(stem4, 4, 512, 1024, 2, (4 * 512 * 1024, 1, 4 * 1024, 4))[0] == 295
    finally:
        K.set_conv_math(K.MATH_F32X3)


def test_workspace_and_kernel_selection_on_host():
    from adaptsegnet_amd import kernels as K
    K.set_conv_math(K.MATH_F32)
    try:
        _fp32_kernel_selection(K)
    finally:
        K.set_conv_math(K.MATH_F32X3)


def _fp32_kernel_selection(K):
    g = K.ConvGeom(256, 256, 3, 3, 1, (2,), (2,))
    kid, splits = K.conv_kernel_id(g, 4, 64, 128, 0)
    assert kid == 84 and splits == 1          # fwd, 128x128 BK16 occupancy-3 tile (cfg 8), FAST, no K split
    kid, splits = K.conv_kernel_id(g, 4, 64, 128, 2)
    assert kid // 100 == 2 and splits > 1     # weight grad splits K = N*OH*OW
    aspp = K.ConvGeom(2048, 19, 3, 3, 1, (6, 12, 18, 24), (6, 12, 18, 24))
    kid, _ = K.conv_kernel_id(aspp, 4, 64, 128, 0)
    assert kid == 84                          # tap-GEMM: the 19-class head runs as a dense
    #                                           1x1 GEMM with N = 36 taps x 19 (pad 704)
    dgrad, _ = K.conv_kernel_id(aspp, 4, 64, 128, 1)
    assert dgrad == 184                       # dX = G * W', K = 704: 1x1 vector data-grad on cfg 8
    kid, _ = K.conv_kernel_id(g, 4, 64, 128, 1)
    assert kid == 104                         # 3x3 stride-1 data grad: 128x128 BK32 tile (cfg 0)
    c1 = K.ConvGeom(1024, 256, 1, 1, 1, (0,), (1,))
    kid, _ = K.conv_kernel_id(c1, 4, 64, 128, 1)
    assert kid == 184                         # 1x1 data grad: occupancy-3 BK16 tile (cfg 8)
    d5 = K.ConvGeom(512, 1, 4, 4, 2, (1,), (1,))  # D classifier (Cout 1): the thin kernels
    kid, _ = K.conv_kernel_id(d5, 4, 32, 64, 0)
    assert kid == 80                          # vector-ALU thin forward
    kid, _ = K.conv_kernel_id(d5, 4, 32, 64, 1)
    assert kid // 100 == 1 and kid % 100 < 80  # stride-2 data grad stays on the implicit GEMM


def test_kernels_use_no_scratch(tmp_path):
    """Every gfx950 kernel in libadaptseg.so runs without private (scratch) memory.  A kernel
    that indexes its ConvParams argument per lane gets the whole struct copied to scratch and
    every global load turned into a flat load (that once cost the fp32 forward conv 40 %)."""
    import re
    import shutil
    import subprocess
    from adaptsegnet_amd import _lib
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not (os.path.exists(objdump) and os.path.exists(readelf)):
        pytest.skip("ROCm LLVM tools not available")
    so = tmp_path / "lib.so"
    shutil.copy(_lib.LIB_PATH, so)
    subprocess.run([objdump, "--offloading", str(so)], check=True, capture_output=True, cwd=tmp_path)
    cos = sorted(tmp_path.glob("lib.so.*gfx950"))
    assert cos, "no gfx950 code object in the library"
    seen = 0
    for co in cos:
        notes = subprocess.run([readelf, "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
        names = re.findall(r"\.name:\s+(\S+)", notes)
        sizes = [int(v) for v in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", notes)]
        assert len(names) == len(sizes)
        bad = [n for n, s in zip(names, sizes) if s != 0]
        assert not bad, f"kernels using scratch: {bad}"
        seen += len(names)
    assert seen > 50


def test_bf16_operand_abi_checks_on_host():
    """The _x entry points (bf16 operand copies): a NULL fp32 operand is accepted only when the
    plan runs a bf16-operand LDS-DMA kernel that reads the copy instead — rejected on the host,
    before any launch, otherwise; and the bf16 selectors of the step's shapes (host planning)."""
    from adaptsegnet_amd import kernels as K
    L = _lib.lib()
    d = K._desc(K.ConvGeom(256, 256, 3, 3, 1, (2,), (2,)), 4, 64, 128, K.nhwc_strides(4, 64, 128, 256))[0]
    w = _lib.ptr_array([16])
    # F32X3 math: the copy is the operand's three term images, which the 256x128x32 kernel reads
    # in place of x (the call passes the host checks and stops at the missing workspace) ...
    st = L.adaptseg_conv2d_fwd_x(ctypes.byref(d), None, ctypes.c_void_p(256), w, None, None, None,
                                 ctypes.c_void_p(512), None, 0, None, 0, None)
    assert st == 4, L.adaptseg_last_error()   # ADAPTSEG_ERR_WORKSPACE
    assert K.conv_kernel_id(K.ConvGeom(256, 256, 3, 3, 1, (2,), (2,)), 4, 64, 128, 0, copies=True)[0] == 88
    # ... but a product that kernel does not cover (Cin 48: a 32-deep step would cross a tap)
    # needs the fp32 input
    d48 = K._desc(K.ConvGeom(48, 64, 3, 3, 1, (1,), (1,)), 4, 64, 128, K.nhwc_strides(4, 64, 128, 48))[0]
    st = L.adaptseg_conv2d_fwd_x(ctypes.byref(d48), None, ctypes.c_void_p(256), w, None, None, None,
                                 ctypes.c_void_p(512), None, 0, None, 0, None)
    assert st == 1 and b"fp32 input" in L.adaptseg_last_error()
    st = L.adaptseg_conv2d_fwd_x(ctypes.byref(d), None, None, w, None, None, None, ctypes.c_void_p(512), None, 0, None,
                                 0, None)
    assert st == 1
    K.set_conv_math(K.MATH_BF16)
    try:
        g = K.ConvGeom(256, 256, 3, 3, 1, (2,), (2,))
        # K 2304, N 256: the 256x256x64 two-stage tile (ADAPTSEG_OPT_G16_WIDE bit 1, the default);
        # bit 2 also puts the weight gradient on the 256x256 tile
        # when its grid has >= 128 tiles (4 x 128 x 128 rows: 256 tiles; 4 x 64 x 128: 128, split K;
        # 4 x 32 x 128: 64, the 128x256 tile)
        assert K.get_g16_wide() == 1
        assert [K.conv_kernel_id(g, 4, 32, 128, op)[0] for op in (0, 1, 2)] == [97, 197, 298]
        assert [K.conv_kernel_id(g, 4, 64, 128, op) for op in (0, 1)] == [(85, 2), (185, 2)]
        assert [K.conv_kernel_id(g, 4, 128, 128, op)[0] for op in (0, 1, 2)] == [85, 185, 298]
        K.set_g16_wide(0)
        assert [K.conv_kernel_id(g, 4, 128, 128, op)[0] for op in (0, 1, 2)] == [97, 197, 298]
        K.set_g16_wide(3)
        assert [K.conv_kernel_id(g, 4, 128, 128, op)[0] for op in (0, 1, 2)] == [85, 185, 285]
        K.set_g16_wide(1)
        s2 = K.ConvGeom(256, 128, 1, 1, 2, (0,), (1,))
        assert K.conv_kernel_id(s2, 4, 128, 256, 1)[0] == 192    # stride-2 parity classes, LDS-DMA
        # weight gradient without the fp32 operands needs both copies (and no bias gradient)
        st = L.adaptseg_conv2d_bwd_weight_x(ctypes.byref(d), None, ctypes.c_void_p(256), None, None,
                                            _lib.ptr_array([1024]), None, 0, None, 0, None)
        assert st == 1
    finally:
        K.set_conv_math(K.MATH_F32X3)


def test_fused_bn_sum_planning_on_host():
    """adaptseg_conv2d_bnsum_tiles (host planning, no GPU): the fused BN backward sums come in one
    partial per output row tile of the data-gradient plan — 128-row tiles on the register-staged
    F32X3 kernel, 256 on the term-image one (with dY's copy) — and none where the plan cannot fuse
    them (a stride-2 parity-class product, a thin one); adaptseg_conv2d_bwd_data_bnsum rejects a
    descriptor without its partial buffer before any launch, and adaptseg_timing_reserve rejects
    a negative count."""
    from adaptsegnet_amd import kernels as K
    L = _lib.lib()
    g1 = K.ConvGeom(256, 64, 1, 1, 1)
    n, h, w = 4, 64, 72
    assert K.conv_bnsum_tiles(g1, n, h, w) == -(-n * h * w // 128)
    g3 = K.ConvGeom(256, 256, 3, 3, 1, (2,), (2,))
    assert K.conv_bnsum_tiles(g3, 2, 96, 96, with_copy=True) == -(-2 * 96 * 96 // 256)
    assert K.conv_bnsum_tiles(K.ConvGeom(64, 128, 3, 3, 2, (1,), (1,)), 2, 64, 64) == 0   # parity classes
    assert K.conv_bnsum_tiles(K.ConvGeom(64, 2, 3, 3, 1, (1,), (1,)), 2, 32, 32) == 0     # thin (Cout 2)
    d = K._desc(g1, n, h, w, K.nhwc_strides(n, h, w, g1.cin))[0]
    bs = _lib.BnSumDesc()
    nt = ctypes.c_int(-1)
    assert L.adaptseg_conv2d_bwd_data_bnsum(ctypes.byref(d), None, None, None, None, None, None, None, None, None, 0,
                                            ctypes.byref(bs), ctypes.byref(nt), None, 0, None) == 1
    assert nt.value == 0 and b"x / x_bf16" in L.adaptseg_last_error()
    assert L.adaptseg_timing_reserve(-1) == 1
    assert L.adaptseg_timing_reserve(0) == 0
