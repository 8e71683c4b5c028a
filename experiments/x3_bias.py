"""Debug: signed (bias) error of F32 vs F32X3 conv products vs fp64, positive and signed data."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch, torch.nn.functional as F
from adaptsegnet_amd import kernels as K
DEV = "cuda"
g = torch.Generator().manual_seed(1)
n, cin, h, w, cout = 2, 256, 32, 48, 256
geom = K.ConvGeom(cin, cout, 3, 3, 1, (1,), (1,))
for kind in ("positive", "signed"):
    x = torch.rand(n, cin, h, w, generator=g, dtype=torch.float64)
    wt = torch.rand(cout, cin, 3, 3, generator=g, dtype=torch.float64) / 2304
    if kind == "signed":
        x = x - 0.5
        wt = wt - 0.5 / 2304
    ref = F.conv2d(x, wt, None, 1, 1)
    gy = torch.rand(ref.shape, generator=g, dtype=torch.float64) - (0.5 if kind == "signed" else 0)
    dref = torch.nn.grad.conv2d_input(x.shape, wt, gy, 1, 1)
    wref = torch.nn.grad.conv2d_weight(x, wt.shape, gy, 1, 1)
    for math in (K.MATH_F32, K.MATH_F32X3):
        K.set_conv_math(math)
        xd = x.permute(0, 2, 3, 1).contiguous().float().to(DEV)
        wd = wt.permute(0, 2, 3, 1).contiguous().float().to(DEV)
        gyd = gy.permute(0, 2, 3, 1).contiguous().float().to(DEV)
        y = K.conv_fwd(geom, xd, n, h, w, [wd]).permute(0, 3, 1, 2).double().cpu()
        dx = K.conv_dgrad(geom, gyd, n, h, w, [wd]).permute(0, 3, 1, 2).double().cpu()
        dw = torch.zeros_like(wd)
        K.conv_wgrad(geom, gyd, xd, n, h, w, [dw], accumulate=False)
        dw = dw.permute(0, 3, 1, 2).double().cpu()
        # the inputs themselves are rounded to fp32: compare against fp64 of the rounded inputs
        xr, wr, gr = x.float().double(), wt.float().double(), gy.float().double()
        r1, r2, r3 = F.conv2d(xr, wr, None, 1, 1), torch.nn.grad.conv2d_input(x.shape, wr, gr, 1, 1), torch.nn.grad.conv2d_weight(xr, wt.shape, gr, 1, 1)
        for nm, a, r in (("fwd", y, r1), ("dgrad", dx, r2), ("wgrad", dw, r3)):
            e = (a - r) / r.abs().max()
            print(f"{kind:8s} math {math} {nm:5s} mean signed err {float(e.mean()):+.2e}  rms {float(e.pow(2).mean().sqrt()):.2e}", flush=True)
K.set_conv_math(K.MATH_F32X3)
