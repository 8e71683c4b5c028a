"""Conv geometries the GPU parity tests run, shared with the CPU coverage test.

A case is (n, cin, h, w, cout, k, stride, pads, dils, bias).  ``case_products`` lists the
(op, kernel selector, split-K?) triples a case exercises, computed by the library's host-side
planner (``adaptseg_conv2d_kernel_id``: no GPU needed), so tests/test_conv_coverage.py can
check that every kernel variant a benchmark step launches is compared with the fp64 oracle
by at least one case.
"""

# fp32 cases of tests/test_ops_gpu.py::test_conv_fwd_dgrad_wgrad (small: most grids split K)
CONV_CASES = [
    (2, 64, 17, 23, 256, 1, 1, (0,), (1,), False),        # bottleneck conv1/conv3 (1x1)
    (2, 256, 17, 23, 128, 1, 2, (0,), (1,), False),       # layer2 stride-2 1x1
    (2, 64, 15, 21, 64, 3, 1, (1,), (1,), False),         # layer1 3x3
    (2, 128, 13, 11, 128, 3, 1, (2,), (2,), False),       # layer3 atrous d2
    (1, 256, 9, 12, 256, 3, 1, (4,), (4,), False),        # layer4 atrous d4
    (2, 3, 37, 45, 64, 7, 2, (3,), (1,), False),          # stem 7x7/2
    (2, 19, 32, 40, 64, 4, 2, (1,), (1,), True),          # D conv1 (Cin 19)
    (2, 20, 32, 40, 64, 4, 2, (1,), (1,), True),          # D conv1 as run: weight gradient at Cin 20
    (2, 4, 37, 45, 64, 7, 2, (3,), (1,), False),          # stem weight gradient on the Cin-4 padded input
    (2, 64, 16, 20, 128, 4, 2, (1,), (1,), True),         # D conv2
    (2, 128, 6, 8, 1, 4, 2, (1,), (1,), True),            # D classifier (Cout 1)
    (2, 64, 7, 9, 19, 3, 1, (6, 12, 18, 24), (6, 12, 18, 24), True),  # ASPP, dil > spatial
    (1, 2048, 3, 5, 7, 1, 1, (0,), (1,), False),          # split-K path (M=15, K=2048)
    (2, 32, 15, 17, 64, 3, 2, (1,), (1,), False),         # stride-2 3x3, odd sizes (parity classes)
    (1, 64, 9, 11, 32, 4, 2, (1,), (1,), True),           # stride-2 4x4, odd sizes
    (3, 64, 20, 24, 64, 3, 1, (1,), (1,), False),         # N = 64 tile (256x64)
    (2, 96, 12, 10, 96, 1, 2, (0,), (1,), False),         # 1x1 stride 2, empty parity classes
    (2, 64, 40, 48, 64, 1, 1, (0,), (1,), True),          # wgrad 64x64 tile, bias Cout 64
    (2, 64, 30, 34, 256, 1, 1, (0,), (1,), False),        # wgrad 256x64 tile (M'=256, N'=64)
    (4, 64, 64, 96, 64, 1, 1, (0,), (1,), True),          # wgrad ~192 K-splits (16-group reduce)
    (1, 32, 8, 10, 320, 1, 1, (0,), (1,), True),          # bias grad with Cout > 256
    (2, 64, 16, 24, 2, 3, 1, (1,), (1,), True),           # thin: the warper's output conv (Cout 2)
    (2, 32, 10, 14, 3, 3, 1, (2,), (2,), False),          # thin: Cout 3, dilated
    (1, 16, 9, 7, 4, 1, 1, (0,), (1,), True),             # thin: Cout 4, 1x1
    (2, 256, 17, 23, 64, 1, 1, (0,), (1,), False),        # 1x1 dgrad on the occupancy-3 BK16 tile, ragged M
    (2, 100, 13, 9, 48, 1, 1, (0,), (1,), False),         # ... ragged N (Cin 100), K = 48 (BK16 but not BK32)
    (1, 1024, 3, 5, 256, 1, 1, (0,), (1,), False),        # ... split-K (M = 15: one row tile)
    (2, 3, 40, 48, 64, 3, 1, (1,), (1,), True),           # DeeplabVGG conv1_1 (Cin 3: per-element wgrad B, 64x64 tile)
    (2, 4, 40, 48, 64, 3, 1, (1,), (1,), True),           # DeeplabVGG conv1_1 weight gradient as run (Cin 4)
]

# Large grids (>= 257 output tiles): forward and data gradient store straight from the
# in-kernel epilogue (splits == 1) — the mode every layer3/4 conv runs in at c2/c3/c5.
# tests/test_ops_gpu.py::test_conv_large_grid_epilogues runs each with the epilogue flags
# the engine uses.
LARGE_CASES = [
    (2, 256, 96, 96, 256, 3, 1, (2,), (2,), False),       # layer3 conv2 (3x3 d2): 288 tiles
    (2, 512, 80, 72, 512, 3, 1, (4,), (4,), False),       # layer4 conv2 (3x3 d4): 360 tiles
    (2, 256, 96, 96, 1024, 1, 1, (0,), (1,), False),      # layer3 conv3 / conv1 (1x1): dgrad on cfg 8
    (2, 64, 192, 192, 64, 3, 1, (1,), (1,), False),       # layer1 conv2 (N = 64: 256x64 tiles)
    (2, 64, 192, 176, 256, 1, 1, (0,), (1,), False),      # layer1 conv3 (1x1 64 -> 256)
    (2, 128, 128, 136, 512, 1, 1, (0,), (1,), False),     # layer2 conv3 (1x1 128 -> 512)
    (2, 64, 256, 272, 128, 4, 2, (1,), (1,), True),       # D conv2 (4x4/2 + bias)
    (2, 1024, 64, 64, 19, 3, 1, (6, 12, 18, 24), (6, 12, 18, 24), True),  # ASPP: tap-GEMM, large inner GEMM
]

# bf16 cases of tests/test_bf16_gpu.py (the kernel covers vector shapes only)
BF16_CASES = [
    (2, 64, 17, 23, 256, 1, 1, (0,), (1,), False),       # 1x1, M and N tails
    (2, 256, 17, 23, 128, 1, 2, (0,), (1,), False),      # stride-2 1x1 (dgrad parity classes)
    (2, 64, 15, 21, 64, 3, 1, (1,), (1,), False),        # 3x3, N = 64 < tile
    (2, 128, 13, 11, 128, 3, 1, (2,), (2,), False),      # atrous d2
    (1, 256, 9, 12, 256, 3, 1, (4,), (4,), False),       # atrous d4
    (2, 64, 16, 20, 128, 4, 2, (1,), (1,), True),        # D conv2 (4x4/2, bias)
    (2, 128, 7, 9, 64, 3, 1, (6, 12, 18, 24), (6, 12, 18, 24), True),  # ASPP segments
    (1, 2048, 3, 5, 64, 1, 1, (0,), (1,), False),        # split-K (M = 15, K = 2048)
    (2, 64, 31, 33, 192, 3, 2, (1,), (1,), False),       # stride-2 3x3, odd sizes
    (4, 64, 64, 96, 64, 1, 1, (0,), (1,), True),         # wgrad, many K splits
    (2, 256, 96, 96, 256, 3, 1, (2,), (2,), False),      # large grid: 288 tiles, no K split
    (2, 256, 96, 96, 1024, 1, 1, (0,), (1,), False),     # large grid 1x1
    (2, 256, 20, 22, 192, 3, 1, (1,), (1,), False),      # LDS-DMA 256x128 tile at K step 64 (fwd)
    (1, 128, 12, 14, 384, 3, 1, (1,), (1,), False),      # dgrad 256x128 / K step 64; wgrad 256-row tile, half-empty
    (2, 128, 19, 25, 128, 3, 2, (1,), (1,), False),      # stride-2 3x3 data gradient, LDS-DMA parity classes 256x128
    (2, 256, 16, 20, 128, 4, 2, (1,), (1,), True),       # D-style 4x4/2 (bias), parity classes on 128x256
    (1, 2048, 86, 256, 768, 1, 1, (0,), (1,), False),    # 256x256x64 two-stage tile, forward (K 2048, 258 tiles)
    (1, 768, 86, 256, 2048, 1, 1, (0,), (1,), False),    # ... data gradient (N 768, K 2048, 258 tiles)
    (1, 2048, 64, 256, 512, 1, 1, (0,), (1,), False),    # ... forward, 128 tiles: split K to 256 blocks
    (1, 512, 64, 256, 2048, 1, 1, (0,), (1,), False),    # ... data gradient, 128 tiles: split K
]


def case_products(k, case, math=None):
    """{(op, selector, split)} for the products a parity test runs on `case`.

    Forward is run on NHWC input and on the NCHW-strided input (the stem path); data and
    weight gradients on NHWC.  `k` is adaptsegnet_amd.kernels; math: the conv math to plan
    under (default: the current one)."""
    n, cin, h, w, cout, ks, stride, pads, dils, _bias = case
    geom = k.ConvGeom(cin, cout, ks, ks, stride, tuple(pads), tuple(dils))
    nchw = (cin * h * w, h * w, w, 1)
    out = set()
    prev = k.get_conv_math()
    if math is not None:
        k.set_conv_math(math)
    try:
        for op, strides in ((0, None), (0, nchw), (1, None), (2, None)):
            sel, sp = k.conv_kernel_id(geom, n, h, w, op, strides)
            out.add((op, sel, sp > 1))
    finally:
        k.set_conv_math(prev)
    return out
