"""How sensitive is the c5 train-BN step to bf16 conv operands — in the REFERENCE's arithmetic?

Runs the oracle (oracle/reference_torch.py: the reference step in stock PyTorch CPU ops) twice
at config c5's geometry (multi-level LS-GAN, source 1280x720, target 1024x512, batch 1): plain
fp32, and with every conv's operands rounded to bf16 (autocast semantics: forward bf16(x) *
bf16(w), data gradient bf16(dy) * bf16(w), weight gradient bf16(dy) * bf16(x), fp32 sums).
Prints the losses and the cosines of the parameter updates.  Result (profiles/r3/
bf16_trainbn_sensitivity.txt): with train-mode BN the trunk update of the bf16 run is
ORTHOGONAL to the fp32 one (cosine -0.002) while the losses agree to 1e-3 and the heads to
0.9998 — the random-init train-BN trunk gradient is chaotic under bf16 rounding, so
tests/test_fullres_gpu.py bounds the c5 train-BN trunk update by the heads / D / losses
instead; with eval-mode BN every group stays above 0.997.
    python experiments/bf16_trainbn_sensitivity.py   (CPU, ~2 min on 8 cores)
"""
import sys, os, time, types
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from oracle import reference_torch as R
torch.set_num_threads(8)

class BfConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil):
        ctx.save_for_backward(x, w); ctx.cfg = (stride, pad, dil); ctx.hasb = b is not None
        xb, wb = x.bfloat16().to(x.dtype), w.bfloat16().to(w.dtype)
        return F.conv2d(xb, wb, b, stride, pad, dil)
    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors; s, p, d = ctx.cfg
        gb = gy.bfloat16().to(gy.dtype); xb = x.bfloat16().to(x.dtype); wb = w.bfloat16().to(w.dtype)
        dx = torch.nn.grad.conv2d_input(x.shape, wb, gb, s, p, d)
        dw = torch.nn.grad.conv2d_weight(xb, w.shape, gb, s, p, d)
        db = gy.sum((0, 2, 3)) if ctx.hasb else None
        return dx, dw, db, None, None, None

def bfconv2d(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    return BfConv.apply(x, w, b, stride, padding, dilation)

def run(bn_train, emulate, geom="c5", dtype=torch.float32):
    src, tgt = (1280, 720), (1024, 512)
    if geom == "small": src, tgt = (57, 41), (49, 33)
    xs = torch.from_numpy(R.det_images((1, 3, src[1], src[0]), 11)).to(dtype)
    lab = torch.from_numpy(R.det_labels((1, src[1], src[0]), 12))
    xt = torch.from_numpy(R.det_images((1, 3, tgt[1], tgt[0]), 13)).to(dtype)
    cfg = dict(level="multi-level", gan="LS", input_size=src, input_size_target=tgt)
    G = R.to_torch(R.det_state(R.g_specs(), 1338), dtype=dtype, trainable=R.g_trainable)
    D1 = R.to_torch(R.det_state(R.d_specs(), 2001), dtype=dtype, trainable=lambda k: True)
    D2 = R.to_torch(R.det_state(R.d_specs(), 2002), dtype=dtype, trainable=lambda k: True)
    opts = R.make_optimizers(G, D1, D2, R.DEFAULT_CFG | cfg)
    old = R.F
    if emulate:
        R.F = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith('__')})
        R.F.conv2d = bfconv2d
    try:
        ref = R.oracle_step(G, D1, D2, opts, cfg, 0, [(xs, lab, xt)], bn_train=bn_train)
    finally:
        R.F = old
    g0 = R.det_state(R.g_specs(), 1338)
    upd = {}
    for k, t in G.items():
        if t.dtype.is_floating_point and t.requires_grad:
            upd[k] = (t.detach().double() - torch.from_numpy(g0[k])).flatten()
    d0 = R.det_state(R.d_specs(), 2002)
    dupd = torch.cat([(D2[k].detach().double() - torch.from_numpy(d0[k])).flatten() for k in D2])
    return ref, upd, dupd

def cos(a, b): return float(F.cosine_similarity(a, b, dim=0))
for bn_train in (True, False):
    t0 = time.time()
    a = run(bn_train, False); b = run(bn_train, True)
    trunk = [k for k in a[1] if not k.startswith(("layer5", "layer6"))]
    heads = [k for k in a[1] if k.startswith(("layer5", "layer6"))]
    ct = cos(torch.cat([a[1][k] for k in trunk]), torch.cat([b[1][k] for k in trunk]))
    ch = cos(torch.cat([a[1][k] for k in heads]), torch.cat([b[1][k] for k in heads]))
    print(f"bn_train={bn_train}: losses fp32 {a[0]} bf16emu {b[0]}")
    print(f"  trunk cos {ct:.5f} heads cos {ch:.5f} D2 cos {cos(a[2], b[2]):.5f}  ({time.time()-t0:.0f}s)")
    # per-layer trunk cosines
    for k in trunk[:6] + trunk[-4:]:
        print("   ", k, f"{cos(a[1][k], b[1][k]):.4f}")
