"""Every conv kernel variant a benchmark step launches is oracle-checked by some GPU case.

Host-side only (the library's planner, ``adaptseg_conv2d_kernel_id``; no GPU): enumerate the
(op, kernel selector, split-K?) triples of one bench step for configs c2 / c3 / c4 / c5
(bench.conv_inventory) and require each to be produced by at least one case of the fp64
parity tests (tests/conv_cases.py: CONV_CASES + LARGE_CASES on fp32 math, BF16_CASES on
bf16).  A kernel variant that only appears at full size (e.g. the in-kernel epilogue of an
unsplit large grid) is exactly what this catches.
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from conv_cases import BF16_CASES, CONV_CASES, LARGE_CASES, case_products  # noqa: E402


def _step_products(config):
    import bench
    from adaptsegnet_amd import kernels as K
    from adaptsegnet_amd.model import DeeplabMulti, DeeplabVGG, FCDiscriminator
    level, _gan, batch, src, tgt, gen, math = bench.CONFIGS[config]
    model = (DeeplabMulti if gen == "DeeplabMulti" else DeeplabVGG)(num_classes=19)
    D = FCDiscriminator(num_classes=19)
    tsize = src if level == "single-level" else tgt
    prods = set()
    prev = K.get_conv_math()
    # bench.CONFIGS "f32": the fp32 configs, which bench.py runs on the default F32X3 maths
    K.set_conv_math(K.MATH_BF16 if math == "bf16" else K.MATH_F32X3)
    try:
        bench.conv_inventory(model, D, level, batch, src, tgt, tsize, products=prods)
    finally:
        K.set_conv_math(prev)
    return prods, math


@pytest.mark.parametrize("config", ["c2", "c3", "c4", "c5"])
def test_every_step_conv_variant_is_oracle_checked(config):
    from adaptsegnet_amd import kernels as K
    prods, math = _step_products(config)
    covered = set()
    if math == "bf16":
        for c in BF16_CASES:
            covered |= case_products(K, c, K.MATH_BF16)
        # products the bf16 kernel does not take (thin / per-element / tap-GEMM) stay on the
        # fp32 kernels, which the fp32 cases cover under bf16 math as well
        for c in CONV_CASES + LARGE_CASES:
            covered |= case_products(K, c, K.MATH_BF16)
    else:   # the fp32 cases run under the three fp32 conv maths (tests/test_ops_gpu.py::conv_math);
        # F32X3_PRESPLIT runs the term-image kernel (conv_x3r.hpp) the F32X3 step uses on the
        # Bottleneck products' operand copies
        for c in CONV_CASES + LARGE_CASES:
            covered |= (case_products(K, c, K.MATH_F32) | case_products(K, c, K.MATH_F32X3) |
                        case_products(K, c, K.MATH_F32X3_PRESPLIT))
    missing = sorted(prods - covered)
    assert not missing, f"{config}: step conv products without an fp64 parity case: {missing}"
