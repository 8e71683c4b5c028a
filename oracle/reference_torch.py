"""TEST INFRASTRUCTURE ONLY — functional CPU restatement of the AdaptSegNet hot path.

Stock PyTorch CPU ops over explicit name->tensor dicts whose keys are the reference's
state_dict keys.  Runs in fp32 or fp64.  Used as the numerical checker for the HIP engine
(tests/, __graft_entry__.smoke) and as the timed CPU baseline of bench.py.  Pinned against
tests/golden/*.npz, which gen_golden.py captured from the reference modules themselves.

Restated reference code (file:line in /root/reference):
  DeeplabMulti / ResNetMulti layout            model/deeplab_multi.py:124-172, 258-260
  Bottleneck.forward                           model/deeplab_multi.py:83-103
  Classifier_Module.forward                    model/deeplab_multi.py:117-121
  ResNetMulti.forward (+ bilinear upsample)    model/deeplab_multi.py:174-194
  get_1x_lr_params_NOscale multiplicity        model/deeplab_multi.py:196-222
  FCDiscriminator.forward                      model/discriminator.py:21-34
  DeeplabVGG layout / forward (c4)             model/deeplab_vgg.py:7-21, 24-49
  CrossEntropy2d.forward                       utils/loss.py:14-36
  step bodies, losses, optimisers, poly LR     train_gta2cityscapes_multi.py:162-177,
                                               355-359, 379-464, 532-546, 570-683
"""
from __future__ import annotations

import warnings

import numpy as np
import torch
import torch.nn.functional as F

# (planes, blocks, stride, dilation) of layer1..layer4 — deeplab_multi.py:137-140, 259
RESNET101 = ((64, 3, 1, 1), (128, 4, 2, 1), (256, 23, 1, 2), (512, 3, 1, 4))
ASPP_RATES = (6, 12, 18, 24)  # deeplab_multi.py:141-142
BN_EPS, BN_MOMENTUM = 1e-5, 0.1


# ---------------------------------------------------------------------------------------
# Parameter specs and deterministic values
# ---------------------------------------------------------------------------------------


def g_specs(num_classes=19, layout=RESNET101):
    """[(state_dict key, shape, kind)] of DeeplabMulti in registration order."""
    out = []

    def conv(key, co, ci, k, bias=False):
        out.append((key + ".weight", (co, ci, k, k), "conv"))
        if bias:
            out.append((key + ".bias", (co,), "bias"))

    def bn(key, c):
        out.extend([(key + ".weight", (c,), "bn_w"), (key + ".bias", (c,), "bn_b"),
                    (key + ".running_mean", (c,), "bn_rm"), (key + ".running_var", (c,), "bn_rv"),
                    (key + ".num_batches_tracked", (), "bn_n")])

    conv("conv1", 64, 3, 7)
    bn("bn1", 64)
    cin = 64
    for li, (planes, nblk, _stride, _dil) in enumerate(layout, 1):
        for b in range(nblk):
            pre = f"layer{li}.{b}."
            bin_ = cin if b == 0 else planes * 4
            conv(pre + "conv1", planes, bin_, 1)
            bn(pre + "bn1", planes)
            conv(pre + "conv2", planes, planes, 3)
            bn(pre + "bn2", planes)
            conv(pre + "conv3", planes * 4, planes, 1)
            bn(pre + "bn3", planes * 4)
            if b == 0:
                conv(pre + "downsample.0", planes * 4, bin_, 1)
                bn(pre + "downsample.1", planes * 4)
        cin = planes * 4
    for li, ci in ((5, 1024), (6, 2048)):
        for r in range(len(ASPP_RATES)):
            conv(f"layer{li}.conv2d_list.{r}", num_classes, ci, 3, bias=True)
    return out


# DeeplabVGG (deeplab_vgg.py:24-43): VGG16 cfg "D" convs with pool4/pool5 removed, conv5
# dilated 2, fc6/fc7 3x3 d4.  (features index, cin, cout, dilation, 2x2 max-pool after ReLU)
VGG_CONVS = ((0, 3, 64, 1, False), (2, 64, 64, 1, True), (5, 64, 128, 1, False),
             (7, 128, 128, 1, True), (10, 128, 256, 1, False), (12, 256, 256, 1, False),
             (14, 256, 256, 1, True), (17, 256, 512, 1, False), (19, 512, 512, 1, False),
             (21, 512, 512, 1, False), (23, 512, 512, 2, False), (25, 512, 512, 2, False),
             (27, 512, 512, 2, False), (29, 512, 1024, 4, False), (31, 1024, 1024, 4, False))


def vgg_specs(num_classes=19):
    """[(key, shape, kind)] of DeeplabVGG in registration order."""
    out = []
    for idx, ci, co, _d, _p in VGG_CONVS:
        out.append((f"features.{idx}.weight", (co, ci, 3, 3), "vconv"))
        out.append((f"features.{idx}.bias", (co,), "vbias"))
    for r in range(4):
        out.append((f"classifier.conv2d_list.{r}.weight", (num_classes, 1024, 3, 3), "conv"))
        out.append((f"classifier.conv2d_list.{r}.bias", (num_classes,), "bias"))
    return out


def vgg_forward(P, x):
    """DeeplabVGG.forward: features (conv+ReLU, 2x2 pools), then Classifier_Module, whose
    ``return`` inside the loop (deeplab_vgg.py:19-21) sums only branches 0 (d6) and 1 (d12)."""
    for idx, _ci, _co, d, pool in VGG_CONVS:
        x = F.relu(F.conv2d(x, P[f"features.{idx}.weight"], P[f"features.{idx}.bias"], 1, d, d))
        if pool:
            x = F.max_pool2d(x, 2, 2)
    out = F.conv2d(x, P["classifier.conv2d_list.0.weight"], P["classifier.conv2d_list.0.bias"], 1, 6, 6)
    return out + F.conv2d(x, P["classifier.conv2d_list.1.weight"], P["classifier.conv2d_list.1.bias"],
                          1, 12, 12)


def d_specs(num_classes=19, ndf=64):
    chans = (num_classes, ndf, ndf * 2, ndf * 4, ndf * 8, 1)
    names = ("conv1", "conv2", "conv3", "conv4", "classifier")
    out = []
    for i, nm in enumerate(names):
        out.append((nm + ".weight", (chans[i + 1], chans[i], 4, 4), "dconv"))
        out.append((nm + ".bias", (chans[i + 1],), "dbias"))
    return out


def det_state(specs, seed, conv_std=0.01, bn_random=True):
    """Deterministic numpy values (PCG64) for every spec; identical on every machine."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for key, shape, kind in specs:
        if kind == "conv":
            v = rng.normal(0.0, conv_std, shape)
        elif kind == "bias":
            fan_in = None
            v = rng.uniform(-0.05, 0.05, shape)
        elif kind == "vconv":  # torchvision VGG: kaiming_normal_(fan_out, relu)
            v = rng.normal(0.0, np.sqrt(2.0 / (shape[0] * shape[2] * shape[3])), shape)
        elif kind == "vbias":
            v = rng.uniform(-0.05, 0.05, shape)
        elif kind in ("dconv", "dbias"):
            wshape = [s for k2, s, kd in specs if k2 == key.rsplit(".", 1)[0] + ".weight"][0]
            bound = 1.0 / np.sqrt(wshape[1] * wshape[2] * wshape[3])
            v = rng.uniform(-bound, bound, shape)
        elif kind == "bn_w":
            v = 1.0 + (0.1 * rng.standard_normal(shape) if bn_random else 0.0 * np.zeros(shape))
        elif kind == "bn_b":
            v = 0.1 * rng.standard_normal(shape) if bn_random else np.zeros(shape)
        elif kind == "bn_rm":
            v = 0.1 * rng.standard_normal(shape) if bn_random else np.zeros(shape)
        elif kind == "bn_rv":
            v = 1.0 + 0.2 * rng.uniform(0, 1, shape) if bn_random else np.ones(shape)
        elif kind == "bn_n":
            v = np.zeros(shape, dtype=np.int64)
        else:  # pragma: no cover
            raise ValueError(kind)
        sd[key] = np.asarray(v, dtype=np.int64 if kind == "bn_n" else np.float64)
    return sd


def det_images(shape, seed):
    """Mean-subtracted BGR-like pixels (train_gta2cityscapes_multi.py:30): U[-122.7, 151]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(-122.7, 151.0, shape)


def det_labels(shape, seed, num_classes=19, ignore_frac=0.1, ignore=255):
    rng = np.random.Generator(np.random.PCG64(seed))
    lab = rng.integers(0, num_classes, shape)
    lab[rng.uniform(0, 1, shape) < ignore_frac] = ignore
    return lab.astype(np.int64)


def to_torch(sd, dtype=torch.float64, trainable=None):
    """numpy state -> torch dict; float entries become leaves (requires_grad per `trainable`)."""
    out = {}
    for k, v in sd.items():
        if v.dtype == np.int64:
            out[k] = torch.from_numpy(v.copy())
        else:
            t = torch.from_numpy(v.copy()).to(dtype)
            if trainable is not None and trainable(k):
                t.requires_grad_(True)
            out[k] = t
    return out


def g_trainable(key):
    """BN affine parameters are frozen (deeplab_multi.py:66-78,131-132,161-162)."""
    if ".running_" in key or key.endswith("num_batches_tracked"):
        return False
    parts = key.split(".")
    mod = parts[-2]
    is_bn = mod.startswith("bn") or (mod == "1" and "downsample" in key)
    return not is_bn


# ---------------------------------------------------------------------------------------
# Forward passes
# ---------------------------------------------------------------------------------------


def _bn(x, P, key, train):
    if train:
        P[key + ".num_batches_tracked"] += 1
    return F.batch_norm(x, P[key + ".running_mean"], P[key + ".running_var"], P[key + ".weight"],
                        P[key + ".bias"], train, BN_MOMENTUM, BN_EPS)


class _StoreBF16(torch.autograd.Function):
    """Round to bf16 (RNE) in the forward: an activation STORED in bf16 (the engine's bf16
    activation storage).  In the backward the gradient w.r.t. it is rounded to bf16 too when
    ``round_grad`` (bf16 gradient storage, engine.lowp_grads: the data / residual gradients of a
    Bottleneck are bf16 tensors), else passed through in full precision."""

    @staticmethod
    def forward(ctx, t, round_grad):
        ctx.round_grad = round_grad
        return t.to(torch.bfloat16).to(t.dtype)

    @staticmethod
    def backward(ctx, g):
        return (g.to(torch.bfloat16).to(g.dtype) if ctx.round_grad else g), None


_ACT_BF16 = [False, False, True]   # activations stored bf16, gradients stored bf16, engine's fp32 exceptions


class bf16_activation_storage:
    """Context manager: inside it, every Bottleneck conv output, BN output and block output is
    rounded to bf16 as it is stored (torch.autocast(bfloat16)'s storage; the engine's config c5
    program, engine.bf16_operands), and with ``grads`` (default) so is the gradient w.r.t. each of
    them (engine.lowp_grads) — except where the engine keeps that gradient in fp32: the output of
    layer4's last block (it comes from the ASPP head's backward) and, when both heads are trained
    (multi-level), the output of layer3's last block (layer4.0's input gradient, which layer5's
    backward accumulates into).  The stem, the classifiers and the discriminators are unaffected,
    as in the engine.

    The exceptions make this oracle model the ENGINE's storage, not torch.autocast's (which would
    round those two gradients as well): ``exceptions=False`` rounds every stored gradient, the
    pure-autocast restatement, and tests/test_oracle_golden.py bounds the gap between the two."""

    def __init__(self, grads=True, exceptions=True):
        self.grads = grads
        self.exceptions = exceptions

    def __enter__(self):
        self._prev = list(_ACT_BF16)
        _ACT_BF16[0], _ACT_BF16[1], _ACT_BF16[2] = True, self.grads, self.exceptions
        return self

    def __exit__(self, *exc):
        _ACT_BF16[:] = self._prev


def _st(t, grad=True):
    return _StoreBF16.apply(t, grad and _ACT_BF16[1]) if _ACT_BF16[0] else t


def _bottleneck(y, P, pre, stride, dil, has_ds, train, out_grad_bf16=True):
    """deeplab_multi.py:83-103 — the stride sits on the first 1x1 conv (:64).  _st: bf16
    storage of each stored activation (identity unless bf16_activation_storage is on);
    out_grad_bf16: the gradient w.r.t. the block output is stored in bf16 too."""
    t = _st(F.conv2d(y, P[pre + "conv1.weight"], None, stride))
    t = _st(F.relu(_bn(t, P, pre + "bn1", train)))
    t = _st(F.conv2d(t, P[pre + "conv2.weight"], None, 1, dil, dil))
    t = _st(F.relu(_bn(t, P, pre + "bn2", train)))
    t = _bn(_st(F.conv2d(t, P[pre + "conv3.weight"])), P, pre + "bn3", train)
    if has_ds:
        sc = _st(_bn(_st(F.conv2d(y, P[pre + "downsample.0.weight"], None, stride)), P,
                     pre + "downsample.1", train))
    else:
        sc = y
    return _st(F.relu(t + sc), out_grad_bf16)


def _aspp(y, P, pre, rates=ASPP_RATES):
    """deeplab_multi.py:117-121: branch 0, then += branches 1..3 (padding = dilation)."""
    out = None
    for r_i, r in enumerate(rates):
        b = F.conv2d(y, P[f"{pre}.conv2d_list.{r_i}.weight"], P[f"{pre}.conv2d_list.{r_i}.bias"],
                     1, r, r)
        out = b if out is None else out + b
    return out


def g_forward(P, x, input_size, train=True, layout=RESNET101, grad_heads=2):
    """ResNetMulti.forward(x, input_size) — deeplab_multi.py:174-194. input_size = (W, H).
    grad_heads: how many heads the caller's loss reaches (1: single-level, pred1 unused) — only
    bf16 gradient storage depends on it (see bf16_activation_storage)."""
    y = F.conv2d(x, P["conv1.weight"], None, 2, 3)
    y = F.relu(_bn(y, P, "bn1", train))
    y = F.max_pool2d(y, 3, 2, 1, ceil_mode=False)
    x1 = None
    for li, (planes, nblk, stride, dil) in enumerate(layout, 1):
        if li == 4:
            x1 = _aspp(y, P, "layer5")
        for b in range(nblk):
            last = b == nblk - 1
            ogb = not (_ACT_BF16[2] and last and (li == 4 or (li == 3 and grad_heads == 2)))
            y = _bottleneck(y, P, f"layer{li}.{b}.", stride if b == 0 else 1, dil, b == 0, train, ogb)
    x2 = _aspp(y, P, "layer6")
    size = (int(input_size[1]), int(input_size[0]))
    up = lambda t: F.interpolate(t, size=size, mode="bilinear", align_corners=True)  # noqa: E731
    return up(x1), up(x2)


def d_forward(Q, x, slope=0.2):
    """FCDiscriminator.forward — discriminator.py:21-34 (4x4/2 convs, LeakyReLU 0.2)."""
    for nm in ("conv1", "conv2", "conv3", "conv4"):
        x = F.leaky_relu(F.conv2d(x, Q[nm + ".weight"], Q[nm + ".bias"], 2, 1), slope)
    return F.conv2d(x, Q["classifier.weight"], Q["classifier.bias"], 2, 1)


# ---------------------------------------------------------------------------------------
# Losses
# ---------------------------------------------------------------------------------------


def cross_entropy2d(predict, target, ignore_label=255, weight=None):
    """utils/loss.py:14-36: keep pixels with 0 <= target != ignore, mean cross entropy."""
    n, c, h, w = predict.shape
    keep = (target >= 0) & (target != ignore_label)
    logits = predict.permute(0, 2, 3, 1)[keep]
    return F.cross_entropy(logits, target[keep], weight=weight)


def adv_loss(d_out, label, gan):
    """BCEWithLogitsLoss / MSELoss against a constant label — train:542-545, 620-624."""
    tgt = torch.full_like(d_out, float(label))
    if gan == "Vanilla":
        return F.binary_cross_entropy_with_logits(d_out, tgt)
    return F.mse_loss(d_out, tgt)


# ---------------------------------------------------------------------------------------
# Optimisers and the step
# ---------------------------------------------------------------------------------------


def lr_poly(base_lr, it, max_iter, power):
    return base_lr * ((1 - float(it) / max_iter) ** power)


def g_param_multiplicity(key):
    """How often get_1x_lr_params_NOscale yields a parameter (deeplab_multi.py:216-222):
    it walks modules() of conv1, bn1, layer1..4 and takes the RECURSIVE parameters() of
    each, so a weight is yielded once per ancestor inside its layerN."""
    if key.startswith("layer5") or key.startswith("layer6") or key == "conv1.weight":
        return 1
    return 4 if ".downsample." in key else 3


def make_optimizers(G, D1, D2, cfg):
    """SGD(optim_parameters) + Adam x2 — train:532-540 (duplicate params, like the reference).
    DeeplabVGG (cfg gen "vgg"): optim_parameters is ``self.parameters()`` (deeplab_vgg.py:53-54),
    one group, so adjust_learning_rate sets only group 0 (train:166-170)."""
    if cfg.get("gen") == "vgg":
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            opt = torch.optim.SGD([t for t in G.values() if t.requires_grad], lr=cfg["learning_rate"],
                                  momentum=cfg["momentum"], weight_decay=cfg["weight_decay"], foreach=False)
        return opt, None, torch.optim.Adam([t for t in D2.values() if t.requires_grad],
                                           lr=cfg["learning_rate_D"], betas=(0.9, 0.99), foreach=False)
    g0, g1 = [], []
    for k, t in G.items():
        if not (isinstance(t, torch.Tensor) and t.requires_grad):
            continue
        if k.startswith("layer5") or k.startswith("layer6"):
            g1.append(t)
        else:
            g0.extend([t] * g_param_multiplicity(k))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        opt = torch.optim.SGD([{"params": g0, "lr": cfg["learning_rate"]},
                               {"params": g1, "lr": 10 * cfg["learning_rate"]}],
                              lr=cfg["learning_rate"], momentum=cfg["momentum"],
                              weight_decay=cfg["weight_decay"], foreach=False)
    mk = lambda Q: torch.optim.Adam([t for t in Q.values() if t.requires_grad],  # noqa: E731
                                    lr=cfg["learning_rate_D"], betas=(0.9, 0.99), foreach=False)
    return opt, (mk(D1) if D1 is not None else None), mk(D2)


DEFAULT_CFG = dict(level="single-level", gan="Vanilla", learning_rate=2.5e-4, learning_rate_D=1e-4,
                   momentum=0.9, weight_decay=5e-4, power=0.9, num_steps=250000, lambda_seg=0.1,
                   lambda_adv_target1=2e-4, lambda_adv_target2=1e-3, iter_size=1,
                   input_size=(1024, 512), input_size_target=(1024, 512), target_size="auto")


def _set_rg(Q, flag):
    for t in Q.values():
        t.requires_grad_(flag)


def oracle_step(G, D1, D2, opts, cfg, i_iter, batches, bn_train=True):
    """One iteration of train_gta2cityscapes_multi.py:373-464 (single) or :560-683 (multi).

    Returns a dict of host loss values accumulated like the reference's *_value sums.
    ``bn_train=False`` runs the generator with eval-mode BN (model.eval()).
    """
    opt, opt_d1, opt_d2 = opts
    c = dict(DEFAULT_CFG)
    c.update(cfg)
    vals = {}

    def acc(name, v):
        vals[name] = vals.get(name, 0.0) + float(v)

    opt.zero_grad()
    lr = lr_poly(c["learning_rate"], i_iter, c["num_steps"], c["power"])
    opt.param_groups[0]["lr"] = lr
    if len(opt.param_groups) > 1:   # train:169-170
        opt.param_groups[1]["lr"] = lr * 10
    lr_d = lr_poly(c["learning_rate_D"], i_iter, c["num_steps"], c["power"])
    for o in (opt_d1, opt_d2):
        if o is not None:
            o.zero_grad()
            o.param_groups[0]["lr"] = lr_d
    n_sub = c["iter_size"]
    tmode = c["target_size"]
    if tmode == "auto":
        tmode = "source" if c["level"] == "single-level" else "target"
    tsize = c["input_size"] if tmode == "source" else c["input_size_target"]
    src_lbl, tgt_lbl = 0, 1
    if c.get("gen") == "vgg":   # DeeplabVGG returns one map, upsampled by the caller (interp)
        def fwd(P, x, size, _train):
            return None, F.interpolate(vgg_forward(P, x), size=(size[1], size[0]), mode="bilinear",
                                       align_corners=True)
    else:
        def fwd(P, x, size, train):
            return g_forward(P, x, size, train, grad_heads=1 if c["level"] == "single-level" else 2)
    for images, labels, images_t in batches:
        if c["level"] == "single-level":
            _set_rg(D2, False)
            _, pred2 = fwd(G, images, c["input_size"], bn_train)
            loss_seg2 = F.cross_entropy(pred2, labels, ignore_index=255)
            (loss_seg2 / n_sub).backward()
            acc("loss_seg2", loss_seg2.item() / n_sub)
            _, pred_t2 = fwd(G, images_t, tsize, bn_train)
            l_adv = adv_loss(d_forward(D2, F.softmax(pred_t2, dim=1)), src_lbl, c["gan"])
            (c["lambda_adv_target2"] * l_adv / n_sub).backward()
            acc("loss_adv_target2", l_adv.item() / n_sub)
            _set_rg(D2, True)
            for pred, lbl in ((pred2.detach(), src_lbl), (pred_t2.detach(), tgt_lbl)):
                l_d = adv_loss(d_forward(D2, F.softmax(pred, dim=1)), lbl, c["gan"]) / n_sub / 2
                l_d.backward()
                acc("loss_D2", l_d.item())
        else:
            _set_rg(D1, False)
            _set_rg(D2, False)
            pred1, pred2 = g_forward(G, images, c["input_size"], bn_train)
            loss_seg1 = F.cross_entropy(pred1, labels, ignore_index=255)
            loss_seg2 = F.cross_entropy(pred2, labels, ignore_index=255)
            ((loss_seg2 + c["lambda_seg"] * loss_seg1) / n_sub).backward()
            acc("loss_seg1", loss_seg1.item() / n_sub)
            acc("loss_seg2", loss_seg2.item() / n_sub)
            pt1, pt2 = g_forward(G, images_t, tsize, bn_train)
            a1 = adv_loss(d_forward(D1, F.softmax(pt1, dim=1)), src_lbl, c["gan"])
            a2 = adv_loss(d_forward(D2, F.softmax(pt2, dim=1)), src_lbl, c["gan"])
            ((c["lambda_adv_target1"] * a1 + c["lambda_adv_target2"] * a2) / n_sub).backward()
            acc("loss_adv_target1", a1.item() / n_sub)
            acc("loss_adv_target2", a2.item() / n_sub)
            _set_rg(D1, True)
            _set_rg(D2, True)
            for (p1, p2), lbl in (((pred1.detach(), pred2.detach()), src_lbl),
                                  ((pt1.detach(), pt2.detach()), tgt_lbl)):
                l1 = adv_loss(d_forward(D1, F.softmax(p1, dim=1)), lbl, c["gan"]) / n_sub / 2
                l2 = adv_loss(d_forward(D2, F.softmax(p2, dim=1)), lbl, c["gan"]) / n_sub / 2
                l1.backward()
                l2.backward()
                acc("loss_D1", l1.item())
                acc("loss_D2", l2.item())
    opt.step()
    if opt_d1 is not None:
        opt_d1.step()
    opt_d2.step()
    return vals
