"""GPU parity of the bf16-MFMA conv path (adaptseg_conv_set_math(BF16), BASELINE config c5).

Semantics (torch.autocast(bfloat16) conv): each product's two operands are rounded to bf16
(round-to-nearest-even), multiplied exactly and accumulated in fp32.  The oracle therefore
rounds the same operands to bf16 on the host and convolves them in fp64, so the only
remaining difference is fp32 accumulation order: max|err| <= 2e-5 * max|ref| (as the fp32
path).  Against the UNROUNDED fp64 conv the error is the bf16 input rounding itself
(~2^-9 relative per operand), checked loosely (<= 2e-2) to show the result is a conv at all.
"""

import os
import sys

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_cases import BF16_CASES  # noqa: E402  (n, cin, h, w, cout, k, stride, pads, dils, bias)


def K():
    from adaptsegnet_amd import kernels
    return kernels


@pytest.fixture
def bf16_math():
    k = K()
    k.set_conv_math(k.MATH_BF16)
    yield k
    k.set_conv_math(k.MATH_F32X3)   # the library default


@pytest.fixture(params=["bf16", "bf16_wide"])
def bf16_any(request):
    """Both bf16 conv maths: the default 128x128 tile and the 128x256 tile (MATH_BF16_WIDE)."""
    k = K()
    k.set_conv_math(k.MATH_BF16 if request.param == "bf16" else k.MATH_BF16_WIDE)
    yield k
    k.set_conv_math(k.MATH_F32X3)   # the library default


def bf(t):
    return t.to(torch.bfloat16).double()


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous().float().to(DEV)


def nchw(t):
    return t.permute(0, 3, 1, 2).double().cpu()


def _ref(x, ws, bs, stride, pads, dils):
    out = None
    for i, (p, d) in enumerate(zip(pads, dils)):
        y = F.conv2d(x, ws[i], bs[i] if bs is not None else None, stride, p, d)
        out = y if out is None else out + y
    return out


@pytest.mark.parametrize("case", BF16_CASES, ids=[f"b{i}" for i in range(len(BF16_CASES))])
def test_bf16_conv_products(case, bf16_any):
    k = bf16_any
    n, cin, h, w, cout, ks, stride, pads, dils, bias = case
    g = torch.Generator().manual_seed(1000 + BF16_CASES.index(case))
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    nseg = len(pads)
    ws = [torch.randn(cout, cin, ks, ks, generator=g, dtype=torch.float64) * 0.1 for _ in range(nseg)]
    bs = [torch.randn(cout, generator=g, dtype=torch.float64) for _ in range(nseg)] if bias else None
    geom = k.ConvGeom(cin, cout, ks, ks, stride, pads, dils)
    oh, ow = geom.out_hw(h, w)
    gy = torch.randn(n, cout, oh, ow, generator=g, dtype=torch.float64)

    # the bf16 kernel must be the one selected (kernel id 100*op + 90 + s2 + 2*(tile width 256))
    for op in (0, 1, 2):
        kid, _ = k.conv_kernel_id(geom, n, h, w, op)
        assert kid // 10 % 10 == 9 or kid % 100 == 85, (op, kid)   # (85: the 256x256x64 bf16 tile)
        if k.get_conv_math() == k.MATH_BF16_WIDE and op < 2 and (cout if op == 0 else cin) >= 256:
            assert kid % 10 >= 2, (op, kid)   # the 256-wide tile

    xd, gyd = nhwc(x), nhwc(gy)
    wd = [t.permute(0, 2, 3, 1).contiguous().float().to(DEV) for t in ws]
    bd = [t.float().to(DEV) for t in bs] if bias else None

    # forward: bf16(x) * bf16(w)
    y = nchw(k.conv_fwd(geom, xd, n, h, w, wd, bd))
    ref = _ref(bf(x), [bf(t) for t in ws], bs, stride, pads, dils)
    assert rel(y, ref) < 2e-5
    assert rel(y, _ref(x, ws, bs, stride, pads, dils)) < 2e-2

    # data gradient: bf16(dy) * bf16(w)
    xr = bf(x).requires_grad_(True)
    _ref(xr, [bf(t) for t in ws], None, stride, pads, dils).backward(bf(gy))
    dx = nchw(k.conv_dgrad(geom, gyd, n, h, w, wd))
    assert rel(dx, xr.grad) < 2e-5

    # weight gradient: bf16(dy) * bf16(x); bias gradient stays an fp32 sum of dy
    wr = [bf(t).requires_grad_(True) for t in ws]
    _ref(bf(x), wr, None, stride, pads, dils).backward(bf(gy))
    dws = [torch.zeros_like(t) for t in wd]
    dbs = [torch.zeros(cout, device=DEV) for _ in range(nseg)] if bias else None
    k.conv_wgrad(geom, gyd, xd, n, h, w, dws, dbs, accumulate=False)
    for i in range(nseg):
        assert rel(dws[i].permute(0, 3, 1, 2).cpu(), wr[i].grad) < 2e-5
        if bias:
            assert rel(dbs[i].cpu(), gy.sum((0, 2, 3))) < 1e-5


def test_bf16_fused_bn_statistics(bf16_math):
    """The bf16 forward also emits the per-row-tile BN statistics of its output."""
    k = bf16_math
    n, cin, h, w, cout = 4, 128, 96, 96, 256   # 288 row tiles: no K split, so statistics are fused
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) * 0.1
    geom = k.ConvGeom(cin, cout, 3, 3, 1, (1,), (1,))
    y, st = k.conv_fwd_bnstats(geom, nhwc(x), n, h, w, [wt.permute(0, 2, 3, 1).contiguous().float().to(DEV)])
    assert st is not None
    ref = F.conv2d(bf(x), bf(wt), None, 1, 1)
    assert rel(nchw(y), ref) < 2e-5
    stats, nt = st
    s = stats.double().cpu()
    cnt = s[:nt]
    means = s[nt:nt + cout * nt].view(cout, nt)
    mean = (means * cnt).sum(1) / cnt.sum()
    assert rel(mean, ref.mean((0, 2, 3))) < 1e-4


def test_bf16_math_is_process_wide_and_default_off():
    k = K()
    assert k.get_conv_math() == k.MATH_F32X3
    geom = k.ConvGeom(64, 64, 3, 3, 1, (1,), (1,))
    kid, _ = k.conv_kernel_id(geom, 2, 16, 16, 0)
    assert kid % 100 in (86, 87, 88, 89, 95, 96)   # an F32X3 kernel, not a bf16-operand one (90..99)
    with pytest.raises(RuntimeError):
        k.set_conv_math(7)


def test_c5_multilevel_ls_step_bf16(bf16_math):
    """Config c5's step (multi-level, LS-GAN) with bf16 conv math, eval-mode BN (well
    conditioned) against the fp64 oracle: every loss of 3 iterations within 2e-2 relative
    (bf16 operand rounding, ~2^-9 per operand, through ~100 layers), and the generator's
    parameter update within cosine 0.99 of the fp64 update.  The per-product semantics are
    pinned tightly by test_bf16_conv_products; this checks the whole program runs on them."""
    import os
    from test_model_gpu import _oracle_run, _run_hip, _groups, _updates, frob, R
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    xs = torch.from_numpy(R.det_images((2, 3, 41, 57), 11))
    lab = torch.from_numpy(R.det_labels((2, 41, 57), 12))
    xt = torch.from_numpy(R.det_images((2, 3, 33, 49), 13))
    data = (xs, lab, xt)
    cfg = dict(level="multi-level", gan="LS", input_size=(57, 41), input_size_target=(49, 33))
    G, _, _, ref = _oracle_run("multi-level", "LS", cfg, data, torch.float64, 3, bn_train=False)
    m, _, _, got = _run_hip("multi-level", "LS", cfg, data, 3, bn_train=False)
    for it in range(3):
        for key, v in ref[it].items():
            print(f"bf16 iter{it} {key}: hip={got[it][key]:.6f} fp64={v:.6f}")
            assert abs(got[it][key] - v) <= 2e-2 * abs(v) + 1e-6, (it, key, got[it][key], v)
    g0 = R.det_state(R.g_specs(), 1338)
    sd = m.state_dict()
    for gname, keys in _groups(G, "multi-level").items():
        f, c = frob(_updates(None, keys, g0, sd), _updates(G, keys, g0))
        print(f"bf16 {gname} update: rel-frob {f:.3e} cos {c:.6f}")
        assert c >= 0.99, (gname, f, c)


def test_bf16_operand_copies_are_bitwise_neutral(bf16_math):
    """The BN passes' bf16 copies (bn_* bf16_out) equal y.to(bfloat16) exactly, and a conv fed
    the copy (conv_fwd / conv_dgrad ``xb`` / ``dyb``: the LDS-DMA kernel reads it instead of
    converting the fp32 operand itself) returns bitwise the result of the plain call."""
    k = bf16_math
    g = torch.Generator().manual_seed(21)
    n, h, w, c, cout = 2, 24, 40, 128, 256
    geom = k.ConvGeom(c, cout, 3, 3, 1, (2,), (2,))
    x = torch.randn(n, h, w, c, generator=g).to(DEV)
    bw, bb = torch.randn(c, generator=g).to(DEV), torch.randn(c, generator=g).to(DEV)
    rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
    y, mean, invstd, yb = k.bn_fwd_train(x, bw, bb, rm, rv, 0.1, 1e-5, relu=True, bf16_out=True)
    assert torch.equal(yb, y.to(torch.bfloat16))
    yi, ybi = k.bn_fwd_infer(x, bw, bb, rm, rv, 1e-5, relu=True, bf16_out=True)
    assert torch.equal(ybi, yi.to(torch.bfloat16))
    wt = [(torch.randn(cout, 3, 3, c, generator=g) * 0.05).to(DEV)]
    kid, sp = k.conv_kernel_id(geom, n, h, w, 0)
    assert kid % 100 in (85, 94, 97, 98, 99), kid   # the LDS-DMA kernel
    assert torch.equal(k.conv_fwd(geom, y, n, h, w, wt, xb=yb), k.conv_fwd(geom, y, n, h, w, wt))
    gy = torch.randn(n, h, w, cout, generator=g).to(DEV)
    dx, dxb = k.bn_bwd(gy, None, x if cout == c else torch.randn(n, h, w, cout, generator=g).to(DEV),
                       torch.ones(cout, device=DEV), torch.zeros(cout, device=DEV), torch.ones(cout, device=DEV),
                       relu=False, train=False, bf16_out=True)
    assert torch.equal(dxb, dx.to(torch.bfloat16))
    assert torch.equal(k.conv_dgrad(geom, dx, n, h, w, wt, dyb=dxb), k.conv_dgrad(geom, dx, n, h, w, wt))
    # weight gradient on bf16 copies of both operands: bitwise the plain call's result
    assert k.conv_kernel_id(geom, n, h, w, 2)[0] % 100 in (85, 98)   # the LDS-DMA weight-gradient kernel, BM 256
    dw0 = [torch.zeros_like(wt[0])]
    dw1 = [torch.zeros_like(wt[0])]
    k.conv_wgrad(geom, gy, y, n, h, w, dw0, accumulate=False)
    k.conv_wgrad(geom, gy, y, n, h, w, dw1, accumulate=False, dyb=gy.to(torch.bfloat16), xb=yb)
    assert torch.equal(dw0[0], dw1[0])


def test_bf16_train_step_skipping_fp32_copies_is_bitwise_neutral(bf16_math, monkeypatch):
    """Train-mode BN under the bf16 conv math: the BN passes whose outputs feed only
    bf16-operand kernels write only the bf16 copy (engine.bf16_only).  Two iterations of the
    multi-level LS step with and without that skipping give bitwise the same losses and
    parameters (the skipped fp32 tensors are never read)."""
    from test_model_gpu import _run_hip, R
    from adaptsegnet_amd import engine
    xs = torch.from_numpy(R.det_images((2, 3, 41, 57), 11))
    lab = torch.from_numpy(R.det_labels((2, 41, 57), 12))
    xt = torch.from_numpy(R.det_images((2, 3, 33, 49), 13))
    cfg = dict(level="multi-level", gan="LS", input_size=(57, 41), input_size_target=(49, 33))
    # the skipping is live on this geometry: layer3's conv2 reads only bf16 copies
    assert engine.bf16_only(bf16_math.ConvGeom(256, 256, 3, 3, 1, (2,), (2,)), 2, 6, 8, (0, 1, 2))
    m_a, d1_a, d2_a, got_a = _run_hip("multi-level", "LS", cfg, (xs, lab, xt), 2, bn_train=True)
    monkeypatch.setattr(engine, "bf16_only", lambda *a, **kw: False)
    m_b, d1_b, d2_b, got_b = _run_hip("multi-level", "LS", cfg, (xs, lab, xt), 2, bn_train=True)
    assert got_a == got_b, (got_a, got_b)
    for ma, mb in ((m_a, m_b), (d1_a, d1_b), (d2_a, d2_b)):
        for (ka, va), (kb, vb) in zip(ma.state_dict().items(), mb.state_dict().items()):
            assert ka == kb and torch.equal(va, vb), ka


@pytest.mark.parametrize("math", ["bf16", "f32x3"])
def test_conv_bf16_output_copy_is_exact(math):
    """conv_fwd / conv_dgrad ``bf16_out``: the epilogue (or split-K reduce, or the separate pass
    of the thin and tap-GEMM paths) writes y.to(bfloat16) exactly beside y (under F32X3: y's three
    RNE terms, pixel-interleaved [..., 3, C], by a pass after the GEMM), and y itself is bitwise
    the plain call's.  The discriminator's conv -> LeakyReLU -> conv chain
    (model/discriminator.py:14-27) feeds these copies to the next conv's _x operand."""
    k = K()

    def copy_of(y):
        if math == "bf16":
            return y.to(torch.bfloat16)
        hi = y.to(torch.bfloat16)
        r = y - hi.float()
        mid = r.to(torch.bfloat16)
        return torch.stack([hi, mid, (r - mid.float()).to(torch.bfloat16)], dim=-2)
    k.set_conv_math(k.MATH_BF16 if math == "bf16" else k.MATH_F32X3)
    try:
        g = torch.Generator().manual_seed(33)
        cases = [  # (n, cin, h, w, cout, ks, stride, pads, dils): D convs (4x4/2), a split-K tail,
            (2, 64, 40, 48, 128, 4, 2, (1,), (1,)),      # thin classifier, the ASPP tap-GEMM shape
            (2, 128, 20, 24, 256, 4, 2, (1,), (1,)),
            (1, 256, 5, 6, 512, 4, 2, (1,), (1,)),
            (2, 512, 9, 11, 1, 4, 1, (1,), (1,)),
            (1, 2048, 9, 11, 19, 3, 1, (6, 12), (6, 12)),
        ]
        for n, cin, h, w, cout, ks, st, pads, dils in cases:
            geom = k.ConvGeom(cin, cout, ks, ks, st, pads, dils)
            oh, ow = geom.out_hw(h, w)
            x = torch.randn(n, h, w, cin, generator=g).to(DEV)
            wt = [(torch.randn(cout, ks, ks, cin, generator=g) * 0.05).to(DEV) for _ in pads]
            bs = [torch.randn(cout, generator=g).to(DEV) for _ in pads]
            y0 = k.conv_fwd(geom, x, n, h, w, wt, bs, flags=k.EPI_LEAKY)
            y1, yb = k.conv_fwd(geom, x, n, h, w, wt, bs, flags=k.EPI_LEAKY, bf16_out=True)
            assert torch.equal(y0, y1) and torch.equal(yb, copy_of(y1)), (cin, cout)
            gy = torch.randn(n, oh, ow, cout, generator=g).to(DEV)
            aux = torch.randn(n, h, w, cin, generator=g).to(DEV)
            d0 = k.conv_dgrad(geom, gy, n, h, w, wt, aux=aux)
            d1, db = k.conv_dgrad(geom, gy, n, h, w, wt, aux=aux, bf16_out=True)
            assert torch.equal(d0, d1) and torch.equal(db, copy_of(d1)), (cin, cout)
    finally:
        k.set_conv_math(k.MATH_F32X3)


def test_discriminator_bf16_output_copies_are_bitwise_neutral(bf16_math, monkeypatch):
    """The discriminator under the bf16 conv math with and without the epilogue-written operand
    copies (engine._copy_pays): bitwise the same output, input gradient and parameter gradients."""
    from adaptsegnet_amd import engine
    from adaptsegnet_amd.model import FCDiscriminator
    torch.manual_seed(3)
    n, h, w = 2, 65, 97
    x = torch.randn(n, 19, h, w, generator=torch.Generator().manual_seed(4)).softmax(1).to(DEV)
    assert engine._copy_pays(bf16_math.ConvGeom(64, 128, 4, 4, 2, (1,), (1,)), n, 33, 49, (0, 2))

    def run():
        torch.manual_seed(3)
        D = FCDiscriminator(num_classes=19).to(DEV)
        xi = x.clone().requires_grad_(True)
        out = D(xi)
        out.backward(torch.ones_like(out))
        torch.cuda.synchronize()
        return out.detach(), xi.grad, [p.grad.clone() for p in D.parameters()]

    a = run()
    monkeypatch.setattr(engine, "_copy_pays", lambda *args, **kw: False)
    b = run()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for ga, gb in zip(a[2], b[2]):
        assert torch.equal(ga, gb)


def test_aspp_tap_gemm_reads_the_bf16_copy_bitwise(bf16_math):
    """The multi-branch dilated classifier (model/deeplab_multi.py:112-121) on the tap-GEMM path
    with the bf16 copy of its input (the last block's output copy): forward and weight gradient
    bitwise the plain calls', the weight gradient taking ``xb`` alone."""
    k = bf16_math
    g = torch.Generator().manual_seed(41)
    n, h, w, c, cout = 1, 65, 129, 1024, 19
    geom = k.ConvGeom(c, cout, 3, 3, 1, (6, 12, 18, 24), (6, 12, 18, 24))
    x = torch.randn(n, h, w, c, generator=g).to(DEV)
    xb = x.to(torch.bfloat16)
    wt = [(torch.randn(cout, 3, 3, c, generator=g) * 0.02).to(DEV) for _ in range(4)]
    bs = [torch.randn(cout, generator=g).to(DEV) for _ in range(4)]
    assert k.conv_kernel_id(geom, n, h, w, 0)[0] % 100 in (85, 94, 97, 98, 99)   # inner GEMM on the LDS-DMA kernel
    assert torch.equal(k.conv_fwd(geom, x, n, h, w, wt, bs, xb=xb), k.conv_fwd(geom, x, n, h, w, wt, bs))
    gy = torch.randn(n, h, w, cout, generator=g).to(DEV)
    dw0 = [torch.zeros_like(t) for t in wt]
    dw1 = [torch.zeros_like(t) for t in wt]
    k.conv_wgrad(geom, gy, x, n, h, w, dw0, accumulate=False)
    k.conv_wgrad(geom, gy, x, n, h, w, dw1, accumulate=False, xb=xb)
    for a, b in zip(dw0, dw1):
        assert torch.equal(a, b)


# (n, cin, h, w, cout, k, stride, pad, dil): the wide tile takes products with N >= 256, K >= 2048
# and >= 128 tiles of 256x256 (128-255: K split to ~256 blocks); smaller grids keep the 128x256 tile
WIDE_SHAPES = [
    (2, 256, 24, 40, 256, 3, 1, 2, 2),     # layer3 conv2 class, 8 wide tiles: stays on 128x256
    (1, 256, 64, 256, 512, 3, 1, 2, 2),    # forward on the wide tile, 128 tiles: split K
    (1, 256, 86, 256, 768, 3, 1, 2, 2),    # forward on the wide tile (K 2304, 258 tiles)
    (1, 768, 86, 256, 256, 3, 1, 2, 2),    # data gradient on the wide tile (N = Cin 768)
    (1, 2048, 96, 256, 704, 1, 1, 0, 1),   # the ASPP tap-GEMM's inner 1x1 (N 704: a ragged tile)
]


def _wide(n, cin, h, w, cout, ks, op):
    m, nn, kk = n * h * w, (cout if op == 0 else cin), ks * ks * (cin if op == 0 else cout)
    return nn >= 256 and kk >= 2048 and -(-m // 256) * -(-nn // 256) >= 128


@pytest.mark.parametrize("shape", WIDE_SHAPES, ids=[f"w{i}" for i in range(len(WIDE_SHAPES))])
def test_bf16_wide_tile_matches_default_and_oracle(bf16_math, shape):
    """ADAPTSEG_OPT_G16_WIDE: forward / data-gradient products with N >= 256, K >= 2048 and >= 256
    tiles on the 256x256x64 two-stage LDS-DMA tile (selector 100*op + 85; with 128-255 tiles, split K):
    the same k order per output as the
    128x256 tile, so bitwise its result on an unsplit plan, and the bf16-rounded fp64 oracle
    within 2e-5 (model/deeplab_multi.py:70-71, 139-140: the c5 atrous products)."""
    k = bf16_math
    n, cin, h, w, cout, ks, stride, pad, dil = shape
    geom = k.ConvGeom(cin, cout, ks, ks, stride, (pad,), (dil,))
    oh, ow = geom.out_hw(h, w)
    g = torch.Generator().manual_seed(500 + WIDE_SHAPES.index(shape))
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, ks, ks, generator=g, dtype=torch.float64) / (cin * ks * ks) ** 0.5
    gy = torch.randn(n, cout, oh, ow, generator=g, dtype=torch.float64)
    xd, gyd, wd = nhwc(x), nhwc(gy), [wt.permute(0, 2, 3, 1).contiguous().float().to(DEV)]
    w0 = k.get_g16_wide()
    k.set_g16_wide(False)
    try:
        base = [k.conv_kernel_id(geom, n, h, w, op) for op in (0, 1)]
        y0, dx0 = k.conv_fwd(geom, xd, n, h, w, wd), k.conv_dgrad(geom, gyd, n, h, w, wd)
        k.set_g16_wide(True)
        wide = [k.conv_kernel_id(geom, n, h, w, op) for op in (0, 1)]
        y1, dx1 = k.conv_fwd(geom, xd, n, h, w, wd), k.conv_dgrad(geom, gyd, n, h, w, wd)
    finally:
        k.set_g16_wide(w0)
    for op, (sel, sp) in enumerate(wide):
        assert (sel == 100 * op + 85) == _wide(n, cin, h, w, cout, ks, op), (op, sel)
    ref = F.conv2d(bf(x), bf(wt), None, stride, pad, dil)
    assert rel(nchw(y1), ref) < 2e-5
    xr = bf(x).requires_grad_(True)
    F.conv2d(xr, bf(wt), None, stride, pad, dil).backward(bf(gy))
    assert rel(nchw(dx1), xr.grad) < 2e-5
    if base[0][1] == 1 and wide[0][1] == 1:
        assert torch.equal(y0, y1)
    if base[1][1] == 1 and wide[1][1] == 1:
        assert torch.equal(dx0, dx1)
    # weight gradient: 256x256 tiles, 64-pixel K steps (selector 285) when Cout and N >= 256
    wr = bf(wt).requires_grad_(True)
    F.conv2d(bf(x), wr, None, stride, pad, dil).backward(bf(gy))
    dws = []
    for on in (False, True):
        k.set_g16_wide(on)
        try:
            sel, sp = k.conv_kernel_id(geom, n, h, w, 2)
            dw = torch.zeros_like(wd[0])
            k.conv_wgrad(geom, gyd, xd, n, h, w, [dw], accumulate=False)
        finally:
            k.set_g16_wide(w0)
        if on and cout >= 256 and ks * ks * cin >= 256:
            assert sel == 285, sel
        assert rel(dw.permute(0, 3, 1, 2).cpu(), wr.grad) < 2e-5
        dws.append((dw, sp))
    if dws[0][1] == 1 and dws[1][1] == 1:
        assert torch.equal(dws[0][0], dws[1][0])
