"""Forward/backward programs of the DeeplabMulti generator and FCDiscriminator on the HIP kernels.

Each public model (``model/deeplab_multi.py``, ``model/discriminator.py``) is ONE
``torch.autograd.Function`` whose forward runs the whole network as a fixed program of
native launches and whose backward replays it in reverse.  Owning the whole backward lets
the engine

* write weight gradients straight into the flat gradient arena (no per-parameter
  AccumulateGrad adds),
* fold residual-gradient sums into the data-gradient epilogue (``EPI_RESIDUAL`` /
  ``EPI_ACCUMULATE``) and run BN backward in place, and
* release each block's saved activations as soon as its backward is done.

Reference semantics followed (file:line in /root/reference):
  Bottleneck.forward                     model/deeplab_multi.py:83-103
  Classifier_Module.forward (ASPP sum)   model/deeplab_multi.py:117-121
  ResNetMulti.forward                    model/deeplab_multi.py:174-194
  FCDiscriminator.forward                model/discriminator.py:21-34
  DeeplabVGG.forward (+ 2-branch ASPP)   model/deeplab_vgg.py:17-21, 46-49
"""
from __future__ import annotations

import dataclasses
import os as _os

import torch

from . import kernels as K

# ---------------------------------------------------------------------------------------
# Weight gradients on a side stream
# ---------------------------------------------------------------------------------------


class WgradStream:
    """Runs weight-gradient GEMMs on a second HIP stream of the same device.

    A weight gradient only depends on its layer's saved input and the data gradient just
    produced on the main stream, and nothing on the main stream depends on it until the
    optimiser; so it overlaps the main stream's chain of data-gradient GEMMs and the
    HBM-bound BN-backward passes.  ``launch`` orders the side stream after everything
    issued so far on the main stream and marks the tensors it reads as used on the side
    stream (the caching allocator then delays their reuse); ``join`` makes the main stream
    wait for every weight gradient before the backward returns.
    """

    _streams: dict = {}

    def __init__(self, device):
        self.main = torch.cuda.current_stream(device)
        side = WgradStream._streams.get(device.index)
        if side is None:
            side = WgradStream._streams[device.index] = WgradStream._new_stream(device)
        self.side = side
        self.used = False

    @staticmethod
    def _new_stream(device):
        """The side stream; ADAPTSEG_WGRAD_CU_MASK="k/d" restricts it to the CUs i with
        i % d < k (adaptseg_stream_create_cu_mask), leaving the rest to the main chain."""
        spec = _os.environ.get("ADAPTSEG_WGRAD_CU_MASK", "")
        if not spec:
            return torch.cuda.Stream(device)
        k, d = (int(v) for v in spec.split("/"))
        with torch.cuda.device(device):
            return torch.cuda.ExternalStream(K.stream_create_cu_mask(k, d), device=device)

    def launch(self, fn, *tensors):
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            fn()
        for t in tensors:
            t.record_stream(self.side)
        self.used = True

    def flush(self):
        """Launch the split-K sums the weight gradients left pending on the side stream
        (DEFER_SPLITK): before anything reads the gradients they write."""
        if self.used and DEFER_SPLITK:
            with torch.cuda.stream(self.side):
                K.splitk_flush()

    def join(self):
        if self.used:
            self.flush()
            self.main.wait_stream(self.side)
            self.used = False


# ---------------------------------------------------------------------------------------
# BatchNorm (train: batch statistics; eval: running statistics)
# ---------------------------------------------------------------------------------------


def bf16_operands() -> bool:
    """Operand copies are on: the BN passes that produce conv operands (BN+ReLU outputs, block
    outputs, BN-backward outputs) write them, and the conv kernels read them instead of the fp32
    tensor (adaptseg_conv2d_*_x); an fp32 tensor is written only where a consumer still reads
    fp32 (bf16_only).
      * BF16 math (config c5): a bf16 copy, which the bf16 LDS-DMA kernels read instead of
        converting the operand themselves.  The generator's activations are also STORED in bf16
        (lowp_storage), as torch.autocast(bfloat16) does.
      * F32X3_PRESPLIT math: the operand's three bf16 terms, pixel-interleaved [..., 3, C]
        (kernels.copies_are_terms), which the 256x128x32 F32X3 kernel (conv_x3r.hpp) reads by
        LDS-DMA instead of splitting fp32 rows in-kernel — the same products, bitwise the same
        results where neither splits K.  Conv outputs stay fp32 (the BN passes read them).  Not
        the default for c2-c4 (F32X3): the term-image kernels are 13 % faster per conv in
        isolation, but one of their blocks fills a CU, so the weight-gradient stream and the
        main chain no longer share CUs, and the BN passes move 6-byte copies — the step measured
        2.4 % slower (profiles/r3/x3_copies_ab.txt)."""
    return K.get_conv_math() in (K.MATH_BF16, K.MATH_BF16_WIDE, K.MATH_F32X3_PRESPLIT)


def lowp_storage() -> bool:
    """bf16 activation storage (the BF16 math only): Bottleneck conv outputs, BN outputs and the
    residual stream are bf16 tensors; BatchNorm normalises them in fp32 with fp32 statistics
    (from the conv's fp32 accumulators); the gradients stay fp32."""
    return K.get_conv_math() in (K.MATH_BF16, K.MATH_BF16_WIDE)


def _switch(name, default, allowed):
    """An A/B environment switch of the production numeric path, checked at import: a value
    outside ``allowed`` (e.g. a mode whose code was removed) raises instead of silently running
    another path.  switches() reports the active values (bench.py records them)."""
    raw = _os.environ.get(name, str(default))
    try:
        v = int(raw)
    except ValueError:
        v = None
    if v not in allowed:
        raise ValueError(f"{name}={raw!r}: supported values are {sorted(allowed)}")
    _SWITCHES[name] = v
    return v


_SWITCHES: dict = {}


def switches() -> dict:
    """The active A/B switch values (environment, read at import)."""
    return dict(_SWITCHES)


# (A/B switch) bf16 gradient storage under the BF16 maths
BF16_GRADS = _switch("ADAPTSEG_BF16_GRADS", 1, (0, 1))

# (A/B switch) the weight gradients' split-K sums deferred to the end of each backward
# (WgradStream.flush, adaptseg.h ADAPTSEG_WGRAD_DEFER_SUM): the same sums, bitwise, launched
# back to back once every weight-gradient GEMM is queued instead of one after each GEMM.
# Measured slower (c2 -1.0 %, c3 -1.4 %, c5 -1.3 %, profiles/r6/splitk_defer_ab.txt): the sums
# still run on the weight-gradient stream, now all at its tail, on slabs that went cold —
# off by default
DEFER_SPLITK = _switch("ADAPTSEG_DEFER_SPLITK", 0, (0, 1))

# (A/B switch) weight gradients on the side stream (WgradStream; 0: inline on the main stream)
WGRAD_STREAM = _switch("ADAPTSEG_WGRAD_STREAM", 1, (0, 1))

# (A/B switch) BN2 + ReLU folded into conv3 (K.OperandBN): where conv3's forward runs on the x3h
# tile and its weight gradient on the register-staged F32X3 kernel (layers 3-4 under the F32X3
# maths), BN2's apply pass is not run — its statistics are finalised alone, conv3's forward and
# weight gradient read BN2's input c2 and apply the BN in their operand gathers (bitwise the
# unfused results) and BN2's backward recomputes its ReLU mask from c2 as before.  Measured slower
# (c2 -1.1 %, c3 -1.1 %, profiles/r6/bn_fold_ab.txt: the x3h forward and the staged weight
# gradient lose more to the in-gather BN than the apply pass cost) — off by default
BN_FOLD = _switch("ADAPTSEG_BN_FOLD", 0, (0, 1, 2, 3))   # bit 1: BN2 -> conv3; bit 2: BN1 -> conv2
_FOLD_OK: dict = {}


def _fold_ok(g, n, h, w) -> bool:
    """conv ``g`` on an n x h x w input can take its operand BN in the forward (with fused
    output statistics) and the weight gradient."""
    key = (g, n, h, w, K.get_conv_math(), K.get_x3h())
    v = _FOLD_OK.get(key)
    if v is None:
        v = _FOLD_OK[key] = (K.operand_bn_ok(g, n, h, w, 0) and K.operand_bn_ok(g, n, h, w, 2) and
                             K.conv_bnstats_tiles(g, n, h, w, K.nhwc_strides(n, h, w, g.cin)) > 0)
    return v


def lowp_grads() -> bool:
    """bf16 GRADIENT storage (the BF16 maths, config c5, with lowp_storage): a Bottleneck's data
    gradients (conv dgrad outputs) and its residual gradient are bf16 tensors, as under
    torch.autocast(bfloat16); BN backward reads them in bf16 and computes in fp32.  Blocks whose
    input gradient feeds an fp32 consumer (the stem's max-pool backward, layer5's ASPP backward
    accumulating into layer4.0's input gradient) write that one in fp32."""
    return lowp_storage() and BF16_GRADS == 1


_BF16_SEL: dict = {}


def bf16_only(g, n, h, w, ops) -> bool:
    """True when every listed product of this conv runs on a kernel that reads only the bf16
    copy of its activation operand (the LDS-DMA kernels; the library's own plan,
    adaptseg_conv2d_copy_operand_only): the fp32 tensor then need not be written at all."""
    for op in ops:
        key = (g, n, h, w, op, K.get_conv_math())
        v = _BF16_SEL.get(key)
        if v is None:
            v = _BF16_SEL[key] = K.conv_copy_operand_only(g, n, h, w, op)
        if not v:
            return False
    return True


def _copy_pays(g, n, h, w, ops) -> bool:
    """True when one of the listed products of conv ``g`` reads a bf16 operand copy, so that
    its producer should write one (the discriminator's conv -> LeakyReLU -> conv chain)."""
    return any(bf16_only(g, n, h, w, (op,)) for op in ops)


def bn_forward_b(bn, x, res, relu, training, tiles=None, bf16=False, fp32=True, ybits=None):
    """bn_forward that also returns the bf16 copy of y (None unless ``bf16``); fp32=False skips
    the fp32 y (returned as None) when every consumer reads the copy.  ybits: a mask_bits_like
    bitmap the pass fills with y's ReLU mask."""
    fp32 = fp32 or not bf16
    if training:
        if tiles is not None:
            r = K.bn_fwd_train_tiles(x, tiles, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                     bn.momentum, bn.eps, res=res, relu=relu, bf16_out=bf16, fp32_out=fp32,
                                     ybits=ybits)
        else:
            r = K.bn_fwd_train(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum,
                               bn.eps, res=res, relu=relu, bf16_out=bf16, fp32_out=fp32, ybits=ybits)
        y, mean, invstd = r[:3]
        return y, (mean, invstd, True), (r[3] if bf16 else None)
    r = K.bn_fwd_infer(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, res=res,
                       relu=relu, bf16_out=bf16, fp32_out=fp32, ybits=ybits)
    y, yb = r if bf16 else (r, None)
    return y, (bn.running_mean, None, False), yb


def bn_forward(bn, x, res, relu, training, tiles=None):
    """tiles: row-tile statistics of x from the producing conv (conv_fwd_bnstats), which
    replace the BN's own statistics pass in train mode."""
    y, st, _ = bn_forward_b(bn, x, res, relu, training, tiles)
    return y, st


def bn_backward(bn, dy, y, x, st, relu, dx=None, dres=None, mask_from_x=False, bf16=False, fp32=True,
                dybits=None, sums=None):
    """mask_from_x: a BN+ReLU without residual recomputes its ReLU mask from x in train
    mode instead of reading the saved output y (one activation read less per pass).
    bf16: return (dx, bf16 copy of dx) for the bf16-math data gradient that consumes dx.
    dybits: a mask bitmap applied to dy first (the Bottleneck's BN3 / downsample BN).
    sums: the backward sums the producing data gradient fused (bn_sums_spec), or None."""
    mean, invstd, train = st
    if not train:  # eval-mode backward needs 1/sqrt(var+eps) of the running statistics
        invstd = torch.rsqrt(bn.running_var + bn.eps)
    elif mask_from_x and relu:
        y = None
    return K.bn_bwd(dy, y, x, bn.weight, mean, invstd, relu=relu, dx=dx, dres=dres, train=train,
                    bias=bn.bias, bf16_out=bf16, fp32_out=fp32 or not bf16, dybits=dybits, sums=sums)


# (A/B switch) the BN backward reduction of a Bottleneck's BN1 / BN2 fused into the epilogue of the
# data gradient that produces its incoming gradient (adaptseg_conv2d_bwd_data_bnsum): the BN
# backward then skips its pass over dy and x.  fp32 gradient storage only (the bf16-output
# epilogue would leave its 16-B store path).  Bit 1: BN2's (conv3's data gradient), bit 2: BN1's
# (conv2's).  Off by default: alone the fused chain is 5 % faster over the c2 shapes
# (tools/bnsum_bench.py), in the step it is slower — c2 -0.9 / -0.8 % (BN2), -0.0 / -0.3 % (BN1),
# -1.0 / -1.3 % (both), c3 within +-0.6 % — because the main chain then reaches the next data
# gradient while the previous product's weight gradient still holds the CUs: the step's GEMM
# kernel time grew 15 ms against 7 ms of BN time removed (profiles/r5/bn_sums_ab.txt).
BN_SUMS = _switch("ADAPTSEG_BN_SUMS", 0, (0, 1, 2, 3))


def bn_sums_spec(bn, x, st, which=3):
    """K.BnSum of a train-mode BN+ReLU (mask recomputed from x) for conv_dgrad(bnsum=...), or None.
    which: the BN_SUMS bit of this BN."""
    mean, invstd, train = st
    if not (BN_SUMS & which and train) or lowp_grads():
        return None
    return K.BnSum(x, mean, invstd, bn.weight, bn.bias, K.BNSUM_RELU_X)


# ---------------------------------------------------------------------------------------
# Bottleneck
# ---------------------------------------------------------------------------------------


class BlockRec:
    __slots__ = ("x", "c1", "y1", "s1", "c2", "y2", "s2", "c3", "s3", "out", "cd", "sd",
                 "n", "h", "w", "oh", "ow", "xb", "y1b", "y2b", "bits3", "abn1", "abn2", "wt2")


# (A/B switch) the Bottleneck's output ReLU mask as a bitmap (1 bit per element) instead of the
# stored block output: BN3's backward and the residual gradient read it
MASK_BITS = _switch("ADAPTSEG_MASK_BITS", 1, (0, 1))


def _conv_bn(g, x, n, h, w, weight, strides=None, xb=None, bf16_only=False):
    """Conv feeding a train-mode BN: also returns the BN's row-tile statistics (or None)."""
    return K.conv_fwd_bnstats(g, x, n, h, w, [weight], strides=strides, xb=xb, bf16_only=bf16_only)


def _conv_plain(g, x, n, h, w, weight, strides=None, xb=None, bf16_only=False):
    return K.conv_fwd(g, x, n, h, w, [weight], strides=strides, xb=xb, bf16_only=bf16_only), None


def x3_forward_terms(g) -> bool:
    """(X3_FWD_TERMS 1; off by default since round 6, the x3h tile reads the fp32 y1 instead)
    F32X3 (default maths, no operand copies): run this conv's forward on the term-image
    kernel (conv_x3r.hpp, 256x128x32 LDS-DMA) with the producing BN writing its input's three
    bf16 terms beside the fp32 tensor — the dilated 3x3 conv2 of layers 3-4 (Cin >= 256).  The
    forward runs without the weight-gradient stream beside it, so the kernel's one-block-per-CU
    footprint costs nothing there (it does in the backward, §3.2).  Same box: c2 26.95 / 26.91
    -> 27.33 / 27.25 images/s, c3 17.35 / 17.36 -> 17.66 / 17.66; extending it to Cin 128 / 64
    (layers 1-2) measured no further gain (profiles/r3/x3r_forward_ab.txt)."""
    return (X3_FWD_TERMS == 1 and K.get_conv_math() == K.MATH_F32X3 and g.kh * g.kw > 1 and g.cin >= 256
            and g.cin % 32 == 0)


# (A/B switch) 1: layers 3-4 conv2 forward on y1's term images (x3r), its backward per
# X3_BWD_TERMS; 0 (default since round 6): no term images — conv2's forward and data gradient run
# on the x3h tile over the fp32 tensors and its weight gradient on the staged kernel.  Same box:
# c2 +1.5 % / +1.1 %, c3 +0.8 % / +0.6 % over the term-image program (two A/B runs,
# profiles/r6/x3_terms_retune_ab.txt): x3h reads 4-B fp32 rows instead of 6-B term images and
# BN1 / BN2's backward write no term copies
X3_FWD_TERMS = _switch("ADAPTSEG_X3_FWD_TERMS", 0, (0, 1))

# (A/B switch) with X3_FWD_TERMS 0: conv2 of Cin >= this (layer 4: 512) keeps its WEIGHT gradient
# on the term-image kernel (x3r_wgrad: 0.54 MFMA alone vs 0.36 for the staged kernel on layer4
# conv2, profiles/r6/pmc/mfma_util_atrous_f32x3.txt) — BN1 writes y1's terms beside the fp32 y1
# and BN2's backward dY2's beside the fp32 dY2, the forward and data gradient stay on x3h.
# 0: off (every conv2 weight gradient on the staged kernel)
X3_WGRAD_TERMS_MIN_C = _switch("ADAPTSEG_X3_WGRAD_TERMS_MIN_C", 512, (0, 256, 512, 1024))


def x3_wgrad_terms(g) -> bool:
    """conv2 ``g``'s weight gradient on term images while its forward reads fp32 (see
    X3_WGRAD_TERMS_MIN_C)."""
    return (X3_WGRAD_TERMS_MIN_C > 0 and not x3_forward_terms(g) and K.get_conv_math() == K.MATH_F32X3
            and g.kh * g.kw > 1 and g.cin >= X3_WGRAD_TERMS_MIN_C and g.cin % 32 == 0)


# (A/B switch) 0: conv2 backward on fp32 operands; 1: its weight gradient on term images (y1's
# from the forward, dY's from BN2's backward); 2 (default): its data gradient too; 3: conv3's data
# and weight gradients too (dY3's terms from BN3's backward, y2's from BN2's forward) — parity
# green, measured c2 -0.7 %, c3 -1.0 % (profiles/r5/x3_conv3_terms_ab.txt; round 4: -0.6..-0.9 %)
X3_BWD_TERMS = _switch("ADAPTSEG_X3_BWD_TERMS", 2, (0, 1, 2, 3))


def block_input_fp32(blk, n, h, w) -> bool:
    """Under bf16 activation storage: does some consumer of this block's INPUT (its conv1 and
    downsample conv: forward and weight gradient) still read fp32?  Then its producer (the
    previous block) writes the fp32 output beside the bf16 one."""
    if not bf16_only(blk.conv1.geom(), n, h, w, (0, 2)):
        return True
    return blk.downsample is not None and not bf16_only(blk.downsample[0].geom(), n, h, w, (0, 2))


def out_fp32_needed(nxt, cls, n, h, w) -> bool:
    """Must a block output of (h, w) also be stored in fp32?  Always, unless bf16 activation
    storage is on; then only when the next Bottleneck ``nxt`` (block_input_fp32) or a classifier
    ``cls`` reading it (its tap-GEMM forward / weight gradient) still reads fp32."""
    if not bf16_operands():
        return True
    if nxt is not None and block_input_fp32(nxt, n, h, w):
        return True
    return cls is not None and not bf16_only(aspp_geom(cls), n, h, w, (0, 2))


def block_forward(blk, x, n, h, w, training, save, xb=None, out_fp32=True):
    """xb: bf16 copy of x (bf16 conv math), or None; x may be None when xb is given (bf16
    activation storage).  out_fp32: also write the fp32 block output (bf16 storage: a consumer
    reads fp32; block_input_fp32).  Returns (out or None, rec, bf16 copy of out)."""
    g1, g2, g3 = blk.conv1.geom(), blk.conv2.geom(), blk.conv3.geom()
    oh, ow = g1.out_hw(h, w)
    conv = _conv_bn if training else _conv_plain
    sh = bf16_operands()   # operand copies (bf16 or F32X3 term images)
    lp = lowp_storage()    # bf16 math: conv outputs stored in bf16
    # y1 / y2 are read only by the next conv's forward and weight gradient (the BN backward
    # recomputes its ReLU mask from x in train mode, reads the bf16 y in eval mode) — with both
    # on bf16-operand kernels, only their bf16 copies are written
    thin1 = sh and bf16_only(g2, n, oh, ow, (0, 2))
    thin2 = sh and bf16_only(g3, n, oh, ow, (0, 2))
    c1, t1 = conv(g1, x, n, h, w, blk.conv1.weight, xb=xb, bf16_only=lp)
    terms2 = not sh and x3_forward_terms(g2)   # conv2's forward on y1's term images
    wt2 = not sh and save and training and x3_wgrad_terms(g2)   # ... or only its weight gradient
    # ... and its weight gradient: then no consumer reads the fp32 y1 (the BN1 backward's ReLU
    # mask comes from x in train mode, from the terms' hi image in eval mode)
    keep1 = terms2 and save and X3_BWD_TERMS >= 1
    need1 = not terms2 or (save and not keep1)
    abn1 = None
    if ((BN_FOLD & 2) and training and not sh and not terms2 and not wt2 and t1 is not None
            and _fold_ok(g2, n, oh, ow) and c1.is_contiguous()):
        # BN1 folded into conv2 (BN_FOLD bit 2): statistics only, y1 never written
        bn1 = blk.bn1
        mean1, is1 = K.bn_fwd_train_tiles_stats(c1, t1, bn1.running_mean, bn1.running_var, bn1.momentum, bn1.eps)
        s1 = (mean1, is1, True)
        abn1 = K.OperandBN(mean1, is1, bn1.weight, bn1.bias)
        y1 = y1b = None
        c2, t2 = K.conv_fwd_bnstats_abn(g2, c1, abn1, n, oh, ow, [blk.conv2.weight])
    else:
        y1, s1, y1b = bn_forward_b(blk.bn1, c1, None, True, training, t1, bf16=sh or terms2 or wt2,
                                   fp32=not thin1 and need1)
        c2, t2 = conv(g2, y1, n, oh, ow, blk.conv2.weight, xb=None if wt2 else y1b, bf16_only=lp)
    # conv3's backward on term images (X3_BWD_TERMS 3): BN2 also writes y2's terms for its weight
    # gradient (the forward still reads the fp32 y2)
    terms3 = not sh and save and X3_BWD_TERMS >= 3 and x3_forward_terms(g2) and g3.cin % 32 == 0
    abn2 = None
    if ((BN_FOLD & 1) and training and not sh and not terms3 and t2 is not None and _fold_ok(g3, n, oh, ow)
            and c2.is_contiguous()):
        # BN2 folded into conv3 (BN_FOLD): statistics only, y2 never written
        bn2 = blk.bn2
        mean2, is2 = K.bn_fwd_train_tiles_stats(c2, t2, bn2.running_mean, bn2.running_var, bn2.momentum, bn2.eps)
        s2 = (mean2, is2, True)
        abn2 = K.OperandBN(mean2, is2, bn2.weight, bn2.bias)
        y2 = y2b = None
        c3, t3 = K.conv_fwd_bnstats_abn(g3, c2, abn2, n, oh, ow, [blk.conv3.weight])
    else:
        y2, s2, y2b = bn_forward_b(blk.bn2, c2, None, True, training, t2, bf16=sh or terms3, fp32=not thin2)
        c3, t3 = conv(g3, y2, n, oh, ow, blk.conv3.weight, xb=y2b, bf16_only=lp)
    cd = sd = None
    if blk.downsample is not None:
        dconv, dbn = blk.downsample[0], blk.downsample[1]
        cd, td = conv(dconv.geom(), x, n, h, w, dconv.weight, xb=xb, bf16_only=lp)
        r, sd, rb = bn_forward_b(dbn, cd, None, False, training, td, bf16=sh, fp32=not sh)
        if sh:
            r = rb   # the residual stream is bf16
    else:
        r = xb if sh else x
    # the output's ReLU mask, out > 0, as a bitmap for the backward (BN3's mask and the residual
    # gradient's): 1 bit per element instead of re-reading the stored output (4 B / 2 B) twice
    # (fp32 storage only: with bf16 storage the output re-read costs 2 B, and the masked residual
    # in the bf16 data-gradient epilogue measured c5 -1.2 %, profiles/r4/mask_bits_ab.txt)
    bits3 = K.mask_bits_like(c3) if (save and MASK_BITS and not lp and g3.cout % 32 == 0) else None
    out, s3, outb = bn_forward_b(blk.bn3, c3, r, True, training, t3, bf16=sh, fp32=not sh or out_fp32,
                                 ybits=bits3)
    rec = None
    if save:
        rec = BlockRec()
        rec.x, rec.c1, rec.y1, rec.s1, rec.c2, rec.y2, rec.s2 = x, c1, y1, s1, c2, y2, s2
        rec.c3, rec.s3, rec.out, rec.cd, rec.sd = c3, s3, (None if bits3 is not None else out), cd, sd
        rec.abn1, rec.abn2 = abn1, abn2
        rec.bits3 = bits3
        rec.n, rec.h, rec.w, rec.oh, rec.ow = n, h, w, oh, ow
        # the weight gradients' operand copies (bf16 / term images) of x, y1, y2
        rec.xb, rec.y1b, rec.y2b = xb, y1b if (sh or keep1 or wt2) else None, y2b
        rec.wt2 = wt2
        if terms3:
            rec.y2 = None   # the backward reads y2's terms (weight gradient, eval-mode mask)
        if sh and bits3 is None:
            rec.out = outb   # bf16 storage: the BN3 backward's mask source is the bf16 output
    return out, rec, outb


def _wgrad(ws, g, dy, x, n, h, w, dws, dbs=None, strides=None, dyb=None, xb=None):
    """Weight gradient of one conv: on the side stream when ``ws`` is given.  dyb / xb: bf16
    copies of both operands (bf16 conv math)."""
    def run():
        K.conv_wgrad(g, dy, x, n, h, w, dws, dbs, strides=strides, dyb=dyb, xb=xb,
                     defer=ws is not None and DEFER_SPLITK == 1)
    if ws is None:
        run()
    else:
        ws.launch(run, *[t for t in (dy, x, dyb, xb) if t is not None])


def _wgrad_abn(ws, g, dy, x_pre, abn, n, h, w, dws):
    """Weight gradient whose x operand is relu(bn(x_pre)) (K.OperandBN), on the side stream when
    ``ws`` is given."""
    def run():
        K.conv_wgrad_abn(g, dy, x_pre, abn, n, h, w, dws)
    if ws is None:
        run()
    else:
        ws.launch(run, *[t for t in (dy, x_pre, abn.mean, abn.invstd) if t is not None])


# ---------------------------------------------------------------------------------------
# Thin input convs (the stem's Cin 3, the discriminator's Cin 19): channel-padded operands
# ---------------------------------------------------------------------------------------
def _round_up(v, m):
    return (v + m - 1) // m * m


def _wgrad_padded(ws, g, dy, x, n, h, w, dw, db=None):
    """Weight gradient of a conv whose Cin is not a multiple of 4 (the stem's 3, D.conv1's 19,
    DeeplabVGG conv1_1's 3): without float4 rows the implicit GEMM falls back to per-element
    gathers (24-30 TF/s).  The NCHW-shaped input ``x`` (any strides) is copied to
    c4 = round_up(Cin, 4) channels (zeros above Cin), the weight gradient runs on the vector /
    F32X3 path into a padded temporary, and its first Cin channels are folded into ``dw``
    (accumulate); ``db`` accumulates directly.  Measured per c2 step: stem 2 x 402 -> 247 µs,
    D.conv1 2 x 701 -> 449 µs (pad copy included).  The forwards stay unpadded: padding
    D.conv1's forward to Cin 32 ran slower (347 -> 533 µs: Cout 64 fills half of the F32X3
    kernel's 128-wide column tile)."""
    c4 = _round_up(g.cin, 4)
    g4 = dataclasses.replace(g, cin=c4)

    def run():
        xp = K.to_nhwc_pad(x, c4)
        dwp = K.zero_(torch.empty((g.cout, g.kh, g.kw, c4), device=dy.device, dtype=torch.float32))
        K.conv_wgrad(g4, dy, xp, n, h, w, [dwp], [db] if db is not None else None,
                     strides=K.nhwc_strides(n, h, w, c4))
        K.to_nhwc_pad(dwp.permute(0, 3, 1, 2)[:, :g.cin], g.cin, out=dw.permute(0, 2, 3, 1), accumulate=True)
    if ws is None:
        run()
    else:
        ws.launch(run, dy, x)


def block_backward(blk, rec, gout, need_w, ws=None, dx_fp32=True):
    """gout: grad of the block output (owned, modified in place; fp32, or bf16 under bf16
    gradient storage).  Returns grad of the input — in fp32 when ``dx_fp32``, else (bf16
    gradient storage) in bf16."""
    n, h, w, oh, ow = rec.n, rec.h, rec.w, rec.oh, rec.ow
    g1, g2, g3 = blk.conv1.geom(), blk.conv2.geom(), blk.conv3.geom()
    # out = relu(bn3(c3) + r): g = gout*[out>0] goes to bn3 and to the residual branch.
    sh = bf16_operands()   # bf16 copies of each data-gradient operand (bf16 conv math)
    # a BN-backward output read only by bf16-operand data / weight gradients: copy only
    f3 = not (sh and bf16_only(g3, n, oh, ow, (1, 2)))
    f2 = not (sh and bf16_only(g2, n, oh, ow, (1, 2)))
    f1 = not (sh and rec.xb is not None and bf16_only(g1, n, h, w, (1, 2)))
    fd = blk.downsample is None or not (sh and rec.xb is not None and
                                        bf16_only(blk.downsample[0].geom(), n, h, w, (1, 2)))
    # bf16 gradient storage: the data gradients are bf16 tensors; a BN backward whose fp32 output
    # is still wanted (f*: a consumer without a bf16-operand kernel) writes it to its own buffer
    lg = lowp_grads()
    bits = rec.bits3
    t3 = not sh and rec.y2b is not None   # F32X3: conv3's backward on term images (X3_BWD_TERMS 3)
    if t3:
        f3 = False
    if bits is not None:   # g = gout * bit: BN3's input gradient; the residual gradient stays implicit
        r = bn_backward(blk.bn3, gout, None, rec.c3, rec.s3, relu=False, dybits=bits, bf16=sh or t3, fp32=f3)
    else:
        r = bn_backward(blk.bn3, gout, rec.out, rec.c3, rec.s3, relu=True, dres=gout, bf16=sh or t3, fp32=f3)
    dc3, dc3b = r if (sh or t3) else (r, None)
    bs2 = bn_sums_spec(blk.bn2, rec.c2, rec.s2, 1)
    r = K.conv_dgrad(g3, dc3, n, oh, ow, [blk.conv3.weight], dyb=dc3b, bf16_only=lg, bnsum=bs2)
    dy2, sums2 = r if bs2 is not None else (r, None)
    if need_w and blk.conv3.weight.grad is not None:
        if rec.abn2 is not None:   # BN2 folded into conv3: its weight gradient reads c2 through BN2
            _wgrad_abn(ws, g3, dc3, rec.c2, rec.abn2, n, oh, ow, [blk.conv3.weight.grad])
        else:
            _wgrad(ws, g3, dc3, rec.y2, n, oh, ow, [blk.conv3.weight.grad], dyb=dc3b, xb=rec.y2b)
    del dc3, dc3b
    # (the saved y is the mask source in eval mode: bf16 like x under bf16 storage)
    # F32X3 (default maths) with y1's term images saved: BN2's backward also writes dY2's terms,
    # and conv2's weight gradient (X3_BWD_TERMS 2: its data gradient too) runs on the
    # term-image kernel (conv_x3r.hpp) instead of splitting both fp32 operands in-kernel
    t2 = not sh and rec.y1b is not None
    if t2 and X3_BWD_TERMS >= 2 and not rec.wt2:   # (wt2: the data gradient reads the fp32 dY2)
        f2 = False
    r = bn_backward(blk.bn2, dy2, rec.y2b if (sh or rec.y2 is None) else rec.y2, rec.c2, rec.s2, relu=True,
                    dx=None if lg else dy2,
                    mask_from_x=True, bf16=sh or t2, fp32=f2, sums=sums2)
    # BN2's output: in place over dy2, or (bf16 gradient storage) a new fp32 tensor / None
    dy2, dy2b = r if (sh or t2) else (r, None)
    if not f2:
        dy2 = None   # not written: its consumers read dy2b
    bs1 = bn_sums_spec(blk.bn1, rec.c1, rec.s1, 2)
    r = K.conv_dgrad(g2, dy2, n, oh, ow, [blk.conv2.weight], dyb=dy2b if (sh or not f2) else None,
                     bf16_only=lg, bnsum=bs1)
    dy1, sums1 = r if bs1 is not None else (r, None)
    if need_w and blk.conv2.weight.grad is not None:
        if rec.abn1 is not None:   # BN1 folded into conv2: its weight gradient reads c1 through BN1
            _wgrad_abn(ws, g2, dy2, rec.c1, rec.abn1, n, oh, ow, [blk.conv2.weight.grad])
        else:
            _wgrad(ws, g2, dy2, rec.y1, n, oh, ow, [blk.conv2.weight.grad], dyb=dy2b, xb=rec.y1b)
    del dy2, dy2b
    r = bn_backward(blk.bn1, dy1, rec.y1b if (sh or rec.y1 is None) else rec.y1, rec.c1, rec.s1, relu=True,
                    dx=None if lg else dy1,
                    mask_from_x=True, bf16=sh, fp32=f1, sums=sums1)
    dy1, dy1b = r if sh else (r, None)
    if not f1:
        dy1 = None
    if need_w and blk.conv1.weight.grad is not None:
        _wgrad(ws, g1, dy1, rec.x, n, h, w, [blk.conv1.weight.grad], dyb=dy1b, xb=rec.xb)
    if blk.downsample is not None:
        dconv, dbn = blk.downsample[0], blk.downsample[1]
        gd = dconv.geom()
        r = bn_backward(dbn, gout, None, rec.cd, rec.sd, relu=False, dx=None if lg else gout, bf16=sh, fp32=fd,
                        dybits=bits)
        goutb = r[1] if sh else None
        gd_in = (r[0] if sh else r) if fd else None   # (gout keeps the residual gradient when not rewritten)
        if need_w and dconv.weight.grad is not None:
            _wgrad(ws, gd, gd_in, rec.x, n, h, w, [dconv.weight.grad], dyb=goutb, xb=rec.xb)
        dx = K.conv_dgrad(gd, gd_in, n, h, w, [dconv.weight], dyb=goutb, bf16_only=lg and not dx_fp32)
        del goutb
        K.conv_dgrad(g1, dy1, n, h, w, [blk.conv1.weight], out=dx, flags=K.EPI_ACCUMULATE, dyb=dy1b)
    elif lg and dx_fp32 != (gout.dtype == torch.float32):
        # identity residual, bf16 gradient storage, the input gradient stored unlike gout
        dx = torch.empty((n, h, w, g1.cin), device=gout.device,
                         dtype=torch.float32 if dx_fp32 else torch.bfloat16)
        K.conv_dgrad(g1, dy1, n, h, w, [blk.conv1.weight], out=dx, res=gout, dyb=dy1b, resbits=bits)
    else:
        # identity residual: dx = dgrad(conv1) + g, written over g in place (g = gout * bit when
        # the mask is a bitmap)
        dx = K.conv_dgrad(g1, dy1, n, h, w, [blk.conv1.weight], out=gout, res=gout, dyb=dy1b, resbits=bits)
    return dx


# ---------------------------------------------------------------------------------------
# ASPP classifier (4 dilated 3x3 branches summed = one 4-segment conv)
# ---------------------------------------------------------------------------------------


def aspp_geom(cls):
    c0 = cls.conv2d_list[0]
    return K.ConvGeom(c0.in_channels, c0.out_channels, 3, 3, 1,
                      tuple(c.padding for c in cls.conv2d_list),
                      tuple(c.dilation for c in cls.conv2d_list))


def aspp_forward(cls, x, n, h, w, xb=None):
    """xb: bf16 copy of x (the last block's output copy, bf16 conv math): the tap-GEMM's inner
    GEMM reads it instead of converting x per call."""
    return K.conv_fwd(aspp_geom(cls), x, n, h, w, [c.weight for c in cls.conv2d_list],
                      [c.bias for c in cls.conv2d_list], xb=xb)


def aspp_backward(cls, gy, x, n, h, w, need_w, gx_out=None, ws=None, xb=None):
    g = aspp_geom(cls)
    if need_w and cls.conv2d_list[0].weight.grad is not None:
        _wgrad(ws, g, gy, x, n, h, w, [c.weight.grad for c in cls.conv2d_list],
               [c.bias.grad for c in cls.conv2d_list], xb=xb)
    if gx_out is None:
        return K.conv_dgrad(g, gy, n, h, w, [c.weight for c in cls.conv2d_list])
    return K.conv_dgrad(g, gy, n, h, w, [c.weight for c in cls.conv2d_list], out=gx_out,
                        flags=K.EPI_ACCUMULATE)


# ---------------------------------------------------------------------------------------
# ResNetMulti
# ---------------------------------------------------------------------------------------


def _input_strides(x):
    # (n, c, h, w) element strides of an NCHW-shaped tensor of any layout
    return tuple(x.stride())


class _DeeplabMultiFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, model, out_h, out_w, save, first_head=True):
        ctx.set_materialize_grads(False)
        training = model.training
        n, c, h, w = x.shape
        xs = _input_strides(x)
        if training:
            K.add_i64(model._bn_counter)
        # stem: conv 7x7/2 -> BN -> ReLU -> maxpool 3x3/2
        gs = model.conv1.geom()
        h0, w0 = gs.out_hw(h, w)
        c0, t0 = (_conv_bn if training else _conv_plain)(gs, x, n, h, w, model.conv1.weight, xs)
        y0, s0 = bn_forward(model.bn1, c0, None, True, training, t0)
        p, am = K.maxpool_fwd(y0)
        ph, pw = p.shape[1], p.shape[2]
        recs = []
        cur, curb, ch, cw = p, None, ph, pw
        blocks = [b for layer in (model.layer1, model.layer2, model.layer3) for b in layer]
        for i, blk in enumerate(blocks):
            nh, nw = blk.conv1.geom().out_hw(ch, cw)
            last = i + 1 == len(blocks)
            nxt = model.layer4[0] if last else blocks[i + 1]
            f32 = out_fp32_needed(nxt, model.layer5 if last else None, n, nh, nw)
            cur, rec, curb = block_forward(blk, cur, n, ch, cw, training, save, xb=curb, out_fp32=f32)
            recs.append(rec)
            ch, cw = nh, nw
        p3, h3, w3 = cur, ch, cw
        p3b = curb
        x1 = aspp_forward(model.layer5, p3, n, h3, w3, xb=p3b) if first_head else None
        q, qb = p3, p3b
        recs4 = []
        n4 = len(model.layer4)
        for i, blk in enumerate(model.layer4):
            last = i + 1 == n4
            f32 = out_fp32_needed(None if last else model.layer4[i + 1], model.layer6 if last else None, n, h3, w3)
            q, rec, qb = block_forward(blk, q, n, h3, w3, training, save, xb=qb, out_fp32=f32)
            recs4.append(rec)
        del curb
        x2 = aspp_forward(model.layer6, q, n, h3, w3, xb=qb)
        x1_up = K.upsample_fwd(x1, out_h, out_w) if first_head else None
        x2_up = K.upsample_fwd(x2, out_h, out_w)
        if save:
            ctx.model = model
            ctx.x = x
            ctx.xs = xs
            ctx.dims = (n, h, w, h0, w0, h3, w3)
            ctx.stem = (c0, y0, s0, am)
            ctx.recs, ctx.recs4 = recs, recs4
            ctx.p3, ctx.q = p3, q
            ctx.p3b, ctx.qb = p3b, qb   # bf16 copies for the classifiers' weight gradients (or None)
            ctx.need_w = anchor.requires_grad
        return (K.as_nchw(x1_up) if first_head else None), K.as_nchw(x2_up)

    @staticmethod
    def backward(ctx, g1_up, g2_up):
        model = ctx.model
        need_w = ctx.need_w
        n, h, w, h0, w0, h3, w3 = ctx.dims
        if need_w:
            idx = list(model._pidx["trunk"])
            if g2_up is not None:
                idx += model._pidx["layer4"] + model._pidx["layer6"]
            if g1_up is not None:
                idx += model._pidx["layer5"]
            model._arena.claim(idx)
        ws = WgradStream(ctx.x.device) if need_w and WGRAD_STREAM else None
        hook = model._grad_hook if need_w else None

        def done(ordinal):
            # a backward unit's weight gradients are queued (on the side stream): the
            # data-parallel hook may start all-reducing the gradient buckets now complete
            # (their deferred split-K sums first)
            if hook is not None:
                if ws is not None:
                    ws.flush()
                hook(ordinal, ws.side if ws is not None else None)

        # unit ordinals follow DeeplabMulti._bwd_units
        n4 = len(model.layer4)
        gp3 = None
        if g2_up is not None:
            gx2 = K.upsample_bwd(K.nhwc_view(g2_up), h3, w3)
            gq = aspp_backward(model.layer6, gx2, ctx.q, n, h3, w3, need_w, ws=ws, xb=ctx.qb)
            done(0)
            del gx2
            ctx.q = ctx.qb = None
            for i in reversed(range(n4)):
                # layer4.0's input gradient is accumulated into by layer5's backward (fp32)
                gq = block_backward(model.layer4[i], ctx.recs4[i], gq, need_w, ws,
                                    dx_fp32=i == 0 and g1_up is not None)
                done(n4 - i)
                ctx.recs4[i] = None
            gp3 = gq
        if g1_up is not None:
            gx1 = K.upsample_bwd(K.nhwc_view(g1_up), h3, w3)
            gp3 = aspp_backward(model.layer5, gx1, ctx.p3, n, h3, w3, need_w, gx_out=gp3, ws=ws, xb=ctx.p3b)
            done(n4 + 1)
            del gx1
        ctx.p3 = ctx.p3b = None
        if gp3 is None:
            done(None)
            if ws is not None:
                ws.join()
            return None, None, None, None, None, None, None
        blocks = [b for layer in (model.layer1, model.layer2, model.layer3) for b in layer]
        g = gp3
        for i in reversed(range(len(blocks))):
            g = block_backward(blocks[i], ctx.recs[i], g, need_w, ws, dx_fp32=i == 0)   # (max-pool backward)
            done(n4 + 2 + len(blocks) - 1 - i)
            ctx.recs[i] = None
        c0, y0, s0, am = ctx.stem
        ctx.stem = None
        dy0 = K.maxpool_bwd(g, am, h0, w0)
        del g
        bn_backward(model.bn1, dy0, y0, c0, s0, relu=True, dx=dy0, mask_from_x=True)
        gs = model.conv1.geom()
        if need_w and model.conv1.weight.grad is not None:
            if gs.cin % 4:   # Cin 3: on a 4-channel padded copy of the input
                _wgrad_padded(ws, gs, dy0, ctx.x, n, h, w, model.conv1.weight.grad)
            else:
                _wgrad(ws, gs, dy0, ctx.x, n, h, w, [model.conv1.weight.grad], strides=ctx.xs)
        done(None)
        dx = None
        if ctx.needs_input_grad[1]:
            dx = K.as_nchw(K.conv_dgrad(gs, dy0, n, h, w, [model.conv1.weight]))
        ctx.x = None
        if ws is not None:
            ws.join()
        return None, dx, None, None, None, None, None


def deeplab_multi_forward(model, x, input_size, first_head=True):
    """ResNetMulti.forward(x, input_size) (model/deeplab_multi.py:174-194) on the HIP engine.
    ``first_head=False``: layer5's head (ASPP + upsample) is skipped, its output None."""
    if not x.is_cuda:
        raise RuntimeError("adaptsegnet_amd DeeplabMulti runs on the HIP engine only; "
                           f"got input on {x.device}")
    if x.dtype != torch.float32:
        raise RuntimeError(f"expected float32 input, got {x.dtype}")
    model._ensure_arena(x.device)
    need_w = any(p.requires_grad for p in model._arena.params)
    grad = torch.is_grad_enabled() and (need_w or x.requires_grad)
    anchor = model._anchors[need_w]
    out_w, out_h = int(input_size[0]), int(input_size[1])
    return _DeeplabMultiFn.apply(anchor, x, model, out_h, out_w, grad, bool(first_head))


# ---------------------------------------------------------------------------------------
# FCDiscriminator
# ---------------------------------------------------------------------------------------


class DiscForward:
    """A discriminator forward kept for a second backward.  The reference runs D twice on the
    same target prediction with the same weights (train_gta2cityscapes_multi.py:423 / :617-618
    for the generator's adversarial loss, :454 / :665-666 for D's own step — D's optimiser steps
    only after both): the second forward recomputes the first bit for bit, so its activations are kept from
    the first (``discriminator_forward(..., keep=)``) and ``discriminator_replay`` returns the
    same output as a new autograd node whose backward yields D's weight gradients."""
    __slots__ = ("acts", "actsb", "dims", "n", "out")

    def __init__(self):
        self.acts = self.actsb = self.dims = self.n = self.out = None

    def tensors(self):
        """Every tensor the replay reads (for record_stream across the step's streams)."""
        ts = [t for t in (self.acts or ()) if t is not None] + [t for t in (self.actsb or ()) if t is not None]
        return ts + ([self.out] if self.out is not None else [])


def _disc_backward(model, acts, actsb, dims, n, gout, need_w, need_dx):
    """The FCDiscriminator backward over saved activations (``acts`` / ``actsb`` are released
    as it goes).  Returns the input gradient (NCHW) when ``need_dx``."""
    convs = model._convs()
    sh = lowp_storage()   # (F32X3 term images would cost the D convs a separate copy pass)
    if need_w:
        model._arena.claim(model._pidx["all"])
    g = K.nhwc_view(gout)
    if not g.is_contiguous():
        g = g.contiguous()
    ws = WgradStream(g.device) if need_w and WGRAD_STREAM else None
    dx, gb = None, None
    for i in reversed(range(len(convs))):
        conv = convs[i]
        geo = conv.geom()
        ch, cw, cs = dims[i]
        if need_w and conv.weight.grad is not None:
            if geo.cin % 4:   # D.conv1 (Cin 19): on a 20-channel padded copy
                _wgrad_padded(ws, geo, g, acts[i], n, ch, cw, conv.weight.grad, conv.bias.grad)
            else:
                _wgrad(ws, geo, g, acts[i], n, ch, cw, [conv.weight.grad], [conv.bias.grad],
                       strides=cs, dyb=gb, xb=actsb[i])
        if i > 0:
            # grad wrt the previous layer's pre-activation: dgrad * leaky'(act)
            ph, pw, _ = dims[i - 1]
            nb = sh and _copy_pays(convs[i - 1].geom(), n, ph, pw, (1, 2) if need_w else (1,))
            r = K.conv_dgrad(geo, g, n, ch, cw, [conv.weight], aux=acts[i], dyb=gb, bf16_out=nb)
            g, gb = r if nb else (r, None)
        elif need_dx:
            dx = K.as_nchw(K.conv_dgrad(geo, g, n, ch, cw, [conv.weight], dyb=gb))
        acts[i] = actsb[i] = None
    if ws is not None:
        ws.join()
    return dx


class _FCDiscriminatorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, model, save, keep=None):
        ctx.set_materialize_grads(False)
        convs = model._convs()
        n, c, h, w = x.shape
        xs = _input_strides(x)
        sh = lowp_storage()   # bf16 math: each conv epilogue also writes the next conv's operand copy
        acts, actsb, dims = [], [], []
        cur, curb, ch, cw, cs = x, None, h, w, xs
        for i, conv in enumerate(convs):
            g = conv.geom()
            last = i == len(convs) - 1
            oh, ow = g.out_hw(ch, cw)
            nb = sh and not last and _copy_pays(convs[i + 1].geom(), n, oh, ow, (0, 2))
            out = K.conv_fwd(g, cur, n, ch, cw, [conv.weight], [conv.bias], strides=cs,
                             flags=0 if last else K.EPI_LEAKY, xb=curb, bf16_out=nb)
            dims.append((ch, cw, cs))
            acts.append(cur)
            actsb.append(curb)
            cur, curb = out if nb else (out, None)
            ch, cw = oh, ow
            cs = K.nhwc_strides(n, ch, cw, g.cout)
        y = K.as_nchw(cur)
        if save:
            ctx.model, ctx.acts, ctx.actsb, ctx.dims, ctx.n = model, acts, actsb, dims, n
            ctx.need_w = anchor.requires_grad
        if keep is not None:   # (own lists: this node's backward releases its entries)
            keep.acts, keep.actsb, keep.dims, keep.n = list(acts), list(actsb), dims, n
            keep.out = y.detach()   # (no reference to the generator's graph through y's grad_fn)
        return y

    @staticmethod
    def backward(ctx, gout):
        if gout is None:
            return None, None, None, None, None
        dx = _disc_backward(ctx.model, ctx.acts, ctx.actsb, ctx.dims, ctx.n, gout, ctx.need_w,
                            ctx.needs_input_grad[1])
        return None, dx, None, None, None


class _DiscReplayFn(torch.autograd.Function):
    """The kept forward's output again, as a node whose backward is D's weight gradients."""

    @staticmethod
    def forward(ctx, anchor, model, keep):
        ctx.set_materialize_grads(False)
        ctx.model, ctx.keep = model, keep
        return keep.out.clone()

    @staticmethod
    def backward(ctx, gout):
        keep = ctx.keep
        if gout is not None:
            _disc_backward(ctx.model, keep.acts, keep.actsb, keep.dims, keep.n, gout, True, False)
        keep.acts = keep.actsb = keep.out = None
        return None, None, None


def discriminator_forward(model, x, keep=None):
    """FCDiscriminator.forward(x) (model/discriminator.py:27-34) on the HIP engine.  ``keep``: a
    DiscForward that receives this forward's activations for ``discriminator_replay``."""
    if not x.is_cuda:
        raise RuntimeError("adaptsegnet_amd FCDiscriminator runs on the HIP engine only; "
                           f"got input on {x.device}")
    model._ensure_arena(x.device)
    need_w = any(p.requires_grad for p in model._arena.params)
    grad = torch.is_grad_enabled() and (need_w or x.requires_grad)
    return _FCDiscriminatorFn.apply(model._anchors[need_w], x, model, grad, keep)


def discriminator_replay(model, keep):
    """The output of the forward ``keep`` holds, bit-identical to running D again on the same
    input with the same weights, whose backward accumulates D's weight gradients (D's parameters
    must require grad by then)."""
    if keep is None or keep.out is None:
        raise RuntimeError("discriminator_replay: no kept forward (or it was replayed already)")
    if not all(p.requires_grad for p in model._arena.params):
        raise RuntimeError("discriminator_replay: D's parameters do not require grad")
    return _DiscReplayFn.apply(model._anchors[True], model, keep)


# ---------------------------------------------------------------------------------------
# DeeplabVGG (model/deeplab_vgg.py:24-51): conv+bias+ReLU stack with 2x2 pools, then the
# two-branch ASPP sum.  ReLU is fused into each conv epilogue; its derivative is applied in
# the next data-gradient epilogue (EPI_RELU_GRAD on the saved post-ReLU activation, which is
# also the pooled value a 2x2 max-pool routes back to).
# ---------------------------------------------------------------------------------------


# (A/B switch) DeeplabVGG (config c4) on F32X3 term images: 0 off; 1 every conv input's and
# every conv output gradient's term images are made (the conv epilogues' / pools' copies) and the
# weight gradients run on the term-image kernel (conv_x3r.hpp); 2 the forwards and data gradients
# read them too
VGG_TERMS = _switch("ADAPTSEG_VGG_TERMS", 2, (0, 1, 2))
# ... only for tensors of at least this many channels (the term images of a conv's input need
# Cin, of its output gradient Cout >= it): the wide late layers, where the term-image kernel's
# weight gradient is 1.5-1.7x the staged one (profiles/r5/conv_shapes_c4_presplit.txt), without
# the 6-B-per-element term copies of the 64- / 128-channel layers at 512x1024 / 256x512.  Same
# box (profiles/r5/vgg_terms_thr_ab.txt): mode 2 at >= 512 channels +1.1 % (41.73 / 41.63 vs
# 41.31 / 41.14 images/s), at >= 1024 +0.7 %, at >= 256 -0.9 %; mode 1 -5 %
VGG_TERMS_MIN_C = _switch("ADAPTSEG_VGG_TERMS_MIN_C", 512, (0, 256, 512, 1024))


def vgg_terms() -> int:
    return VGG_TERMS if K.get_conv_math() == K.MATH_F32X3 else 0


class _DeeplabVGGFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, model, save):
        ctx.set_materialize_grads(False)
        n, c, h, w = x.shape
        prog = model.conv_program()
        vt = vgg_terms()
        acts = []  # (conv input, h, w, strides, pool record or None, input's term images or None)
        cur, ch, cw, cs = x, h, w, _input_strides(x)
        curt = None
        for i, (conv, pool) in enumerate(prog):
            g = conv.geom()
            # the next conv's input terms: from this conv's epilogue, or from the pool after it
            want_t = vt > 0 and save and i + 1 < len(prog) and g.cout % 8 == 0 and g.cout >= VGG_TERMS_MIN_C
            out = K.conv_fwd(g, cur, n, ch, cw, [conv.weight], [conv.bias], strides=cs,
                             flags=K.EPI_RELU, xb=curt if vt >= 2 else None, bf16_out=want_t and not pool)
            outt = None
            if want_t and not pool:
                out, outt = out
            rec = [cur, ch, cw, cs, None, curt]
            ch, cw = g.out_hw(ch, cw)
            if pool:
                ph, pw = ch, cw
                if want_t:
                    cur, am, curt = K.maxpool_fwd(out, k=2, s=2, p=0, terms=True)
                else:
                    cur, am = K.maxpool_fwd(out, k=2, s=2, p=0)
                    curt = None
                rec[4] = (am, ph, pw)
                ch, cw = cur.shape[1], cur.shape[2]
                del out
            else:
                cur, curt = out, outt
            cs = K.nhwc_strides(n, ch, cw, cur.shape[3])
            acts.append(rec)
        branches = model.classifier_branches()
        gc = _branches_geom(branches)
        y = K.conv_fwd(gc, cur, n, ch, cw, [b.weight for b in branches], [b.bias for b in branches])
        if save:
            ctx.model, ctx.acts, ctx.n = model, acts, n
            ctx.cls_in = (cur, ch, cw)
            ctx.need_w = anchor.requires_grad
        return K.as_nchw(y)

    @staticmethod
    def backward(ctx, gout):
        if gout is None:
            return None, None, None, None
        model, acts, n = ctx.model, ctx.acts, ctx.n
        need_w = ctx.need_w
        if need_w:
            model._arena.claim(model._pidx["used"])
        g = K.nhwc_view(gout)
        if not g.is_contiguous():
            g = g.contiguous()
        branches = model.classifier_branches()
        gc = _branches_geom(branches)
        a, ch, cw = ctx.cls_in
        ctx.cls_in = None
        ws = WgradStream(g.device) if need_w and WGRAD_STREAM else None
        if need_w and branches[0].weight.grad is not None:
            _wgrad(ws, gc, g, a, n, ch, cw, [b.weight.grad for b in branches],
                   [b.bias.grad for b in branches])
        # grad of fc7's pre-activation: dgrad * relu'(a) (+ its term images for fc7's products)
        vt = vgg_terms()
        r = K.conv_dgrad(gc, g, n, ch, cw, [b.weight for b in branches], aux=a,
                         flags=K.EPI_RELU_GRAD, bf16_out=vt > 0)
        g, gt = r if vt > 0 else (r, None)
        del a
        prog = model.conv_program()
        dx = None
        for i in reversed(range(len(prog))):
            conv, _ = prog[i]
            geo = conv.geom()
            xin, ih, iw, cs, _, xint = acts[i]
            if need_w and conv.weight.grad is not None:
                if geo.cin % 4:   # conv1_1 (Cin 3): on a 4-channel padded copy
                    _wgrad_padded(ws, geo, g, xin, n, ih, iw, conv.weight.grad, conv.bias.grad)
                else:
                    ok = gt is not None and xint is not None
                    _wgrad(ws, geo, g, xin, n, ih, iw, [conv.weight.grad], [conv.bias.grad], strides=cs,
                           dyb=gt if ok else None, xb=xint if ok else None)
            if i > 0:
                # grad of the previous conv's pre-activation.  xin is its post-ReLU output,
                # or the 2x2 max of it: relu' at the routed (argmax) position = [max > 0].
                prev_pool = acts[i - 1][4]
                # the previous conv's output-gradient terms: from this data gradient's epilogue,
                # or from the pool's backward
                want_t = vt > 0 and i - 1 > 0 and geo.cin % 8 == 0 and geo.cin >= VGG_TERMS_MIN_C
                r = K.conv_dgrad(geo, g, n, ih, iw, [conv.weight], aux=xin, flags=K.EPI_RELU_GRAD,
                                 dyb=gt if vt >= 2 else None, bf16_out=want_t and prev_pool is None)
                g, gt = r if (want_t and prev_pool is None) else (r, None)
                if prev_pool is not None:
                    am, ph, pw = prev_pool
                    if want_t:
                        g, gt = K.maxpool_bwd(g, am, ph, pw, k=2, s=2, p=0, terms=True)
                    else:
                        g = K.maxpool_bwd(g, am, ph, pw, k=2, s=2, p=0)
            elif ctx.needs_input_grad[1]:
                dx = K.as_nchw(K.conv_dgrad(geo, g, n, ih, iw, [conv.weight]))
            acts[i] = None
        if ws is not None:
            ws.join()
        return None, dx, None, None


def _branches_geom(branches):
    c0 = branches[0]
    return K.ConvGeom(c0.in_channels, c0.out_channels, 3, 3, 1,
                      tuple(b.padding for b in branches), tuple(b.dilation for b in branches))


def deeplab_vgg_forward(model, x):
    """DeeplabVGG.forward(x) (model/deeplab_vgg.py:46-49) on the HIP engine."""
    if not x.is_cuda:
        raise RuntimeError("adaptsegnet_amd DeeplabVGG runs on the HIP engine only; "
                           f"got input on {x.device}")
    if x.dtype != torch.float32:
        raise RuntimeError(f"expected float32 input, got {x.dtype}")
    model._ensure_arena(x.device)
    need_w = any(p.requires_grad for p in model._arena.params)
    grad = torch.is_grad_enabled() and (need_w or x.requires_grad)
    return _DeeplabVGGFn.apply(model._anchors[need_w], x, model, grad)


# ---------------------------------------------------------------------------------------
# The fork's Warper (model/warper.py:216-267) and the prediction warp
# (model/deeplab_multi.py:238-255).  Encoder: 4x4/2 convs, LeakyReLU(0.2) fused into the first
# conv's epilogue and into every BN apply (the in-place LeakyReLU of the NEXT block rewrites the
# stored skip, so the skips are post-LeakyReLU); decoder: ReLU + x2 upsample + skip concat in
# one pass (up2_relu_cat), 3x3 conv, BN.  All BNs are train-mode with trainable affine params.
# ---------------------------------------------------------------------------------------


def _warper_pidx(model):
    A = model.arena
    return A.index_of([p for name, p in model.named_parameters()
                       if p.requires_grad and not name.startswith("connection.")])


class _WarperFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, model, save):
        ctx.set_materialize_grads(False)
        training = model.training
        n, c, h, w = x.shape
        xs = _input_strides(x)
        if training:
            K.add_i64(model._bn_counter)
        enc, out_conv = model.encoder_blocks()
        dec, last = model.decoder_blocks()
        conv_bn = _conv_bn if training else _conv_plain
        # encoder: s_k = leaky(bn(conv(s_{k-1}))), s_0 = leaky(conv(x))
        g0 = enc[0][0].geom()
        s = [K.conv_fwd(g0, x, n, h, w, [enc[0][0].weight], strides=xs, flags=K.EPI_LEAKY)]
        hw = [g0.out_hw(h, w)]
        cs, sts = [None], [None]
        for conv, bn in enc[1:]:
            g = conv.geom()
            ch, cw = hw[-1]
            cc, tiles = conv_bn(g, s[-1], n, ch, cw, conv.weight)
            y, st = bn_forward(bn, cc, None, K.ACT_LEAKY, training, tiles)
            s.append(y)
            cs.append(cc)
            sts.append(st)
            hw.append(g.out_hw(ch, cw))
        # The in-place ReLUs of DecoderInput / DecoderOutput rewrite the latent clone and the last
        # decoder BN output that SkipConnectionDecode returns in warp_list (warper.py:130-144):
        # both are produced post-ReLU here (the ReLU epilogue of the latent conv, the BN apply of
        # the last block).  Nothing reads the pre-ReLU values: the next pass applies the ReLU
        # anyway and its backward masks on the same sign.
        go = out_conv.geom()
        latent = K.conv_fwd(go, s[-1], n, hw[-1][0], hw[-1][1], [out_conv.weight], flags=K.EPI_RELU)
        lh, lw = go.out_hw(*hw[-1])
        # decoder: d_i = bn(conv(up2(relu(cat(skip, d_{i-1}))))), skip = s[L-1-i]
        L = len(s) + 1
        us, dcs, ds, dsts = [], [], [], []
        cur, ch, cw = latent, lh, lw
        for i, (conv, bn) in enumerate(dec):
            skip = None if i == 0 else s[L - 1 - i]
            u = K.up2_relu_cat_fwd(skip, cur)
            ch, cw = 2 * ch, 2 * cw
            cc, tiles = conv_bn(conv.geom(), u, n, ch, cw, conv.weight)
            act = K.ACT_RELU if i == len(dec) - 1 else K.ACT_NONE
            y, st = bn_forward(bn, cc, None, act, training, tiles)
            us.append(u)
            dcs.append(cc)
            ds.append(y)
            dsts.append(st)
            cur = y
        u = K.up2_relu_cat_fwd(None, cur)
        us.append(u)
        ch, cw = 2 * ch, 2 * cw
        flow = K.conv_fwd(last.geom(), u, n, ch, cw, [last.weight], [last.bias])
        wl = [K.as_nchw(latent)] + [K.as_nchw(t) for t in ds]
        ctx.mark_non_differentiable(*wl)
        if save:
            ctx.model, ctx.x, ctx.xs, ctx.dims = model, x, xs, (n, h, w)
            ctx.s, ctx.cs, ctx.sts, ctx.hw = s, cs, sts, hw
            ctx.latent, ctx.lhw = latent, (lh, lw)
            ctx.us, ctx.dcs, ctx.ds, ctx.dsts = us, dcs, ds, dsts
            ctx.need_w = anchor.requires_grad
            ctx.training = training
        return (K.as_nchw(flow), *wl)

    @staticmethod
    def backward(ctx, gflow, *_unused):
        nones = (None,) * 4
        if gflow is None:
            return nones
        if not ctx.training:
            raise NotImplementedError("Warper backward is implemented for train-mode BatchNorm "
                                      "(the reference trains it with WarpModel.train(), train:217-220)")
        model, need_w = ctx.model, ctx.need_w
        n, h, w = ctx.dims
        enc, out_conv = model.encoder_blocks()
        dec, last = model.decoder_blocks()
        if need_w:
            model._arena.claim(_warper_pidx(model))
        g = K.nhwc_view(gflow)
        if not g.is_contiguous():
            g = g.contiguous()
        ws = WgradStream(g.device) if need_w and WGRAD_STREAM else None

        def wgrad(conv, dy, xin, hh, ww, strides=None):
            if need_w and conv.weight.grad is not None:
                dbs = [conv.bias.grad] if conv.bias is not None and conv.bias.grad is not None else None
                _wgrad(ws, conv.geom(), dy, xin, n, hh, ww, [conv.weight.grad], dbs, strides=strides)

        def bn_bwd(bn, dy, y, x, st, act):
            mean, invstd, _ = st
            dw = bn.weight.grad if need_w else None
            db = bn.bias.grad if need_w else None
            if dw is None and db is None:
                return K.bn_bwd(dy, y, x, bn.weight, mean, invstd, relu=act, dx=dy, bias=bn.bias)
            return K.bn_bwd_affine(dy, y, x, bn.weight, bn.bias, mean, invstd, act, dw, db, dx=dy)

        s, ds, us = ctx.s, ctx.ds, ctx.us
        L = len(s) + 1
        # DecoderOutput conv (+bias) on u_last at full resolution
        wgrad(last, g, us[-1], h, w)
        du = K.conv_dgrad(last.geom(), g, n, h, w, [last.weight])
        del g
        _, dd = K.up2_relu_cat_bwd(None, ds[-1], du)
        del du
        us[-1] = None
        skip_grads = [None] * len(s)
        for i in reversed(range(len(dec))):
            conv, bn = dec[i]
            uh, uw = ctx.us[i].shape[1], ctx.us[i].shape[2]
            bn_bwd(bn, dd, None, ctx.dcs[i], ctx.dsts[i], K.ACT_NONE)
            wgrad(conv, dd, us[i], uh, uw)
            du = K.conv_dgrad(conv.geom(), dd, n, uh, uw, [conv.weight])
            del dd
            us[i] = ctx.dcs[i] = None
            skip = None if i == 0 else s[L - 1 - i]
            src = ctx.latent if i == 0 else ds[i - 1]
            dskip, dd = K.up2_relu_cat_bwd(skip, src, du)
            del du
            if i > 0:
                skip_grads[L - 1 - i] = dskip
        dlat = dd
        # EncoderOutput conv: its input s[-1] also feeds the first decoder skip
        hh, ww = ctx.hw[-1]
        wgrad(out_conv, dlat, s[-1], hh, ww)
        gk = K.conv_dgrad(out_conv.geom(), dlat, n, hh, ww, [out_conv.weight],
                          out=skip_grads[-1], flags=K.EPI_ACCUMULATE if skip_grads[-1] is not None else 0)
        del dlat
        for k in reversed(range(1, len(s))):
            conv, bn = enc[k]
            bn_bwd(bn, gk, s[k], ctx.cs[k], ctx.sts[k], K.ACT_LEAKY)
            ph, pw = ctx.hw[k - 1]
            wgrad(conv, gk, s[k - 1], ph, pw)
            if k - 1 >= 1:
                prev = skip_grads[k - 1]
                gk = K.conv_dgrad(conv.geom(), gk, n, ph, pw, [conv.weight], out=prev,
                                  flags=K.EPI_ACCUMULATE if prev is not None else 0)
            else:   # s_0 = leaky(conv0(x)): fold leaky'(s_0) into the data-gradient epilogue
                gk = K.conv_dgrad(conv.geom(), gk, n, ph, pw, [conv.weight], aux=s[0])
            ctx.cs[k] = None
        conv0 = enc[0][0]
        wgrad(conv0, gk, ctx.x, h, w, strides=ctx.xs)
        dx = None
        if ctx.needs_input_grad[1]:
            dx = K.as_nchw(K.conv_dgrad(conv0.geom(), gk, n, h, w, [conv0.weight]))
        ctx.x = ctx.s = ctx.latent = None
        if ws is not None:
            ws.join()
        return None, dx, None, None


def warper_forward(model, x):
    """Warper.forward(pose) (model/warper.py:263-267) on the HIP engine -> (flow, warp_list)."""
    if not x.is_cuda:
        raise RuntimeError("adaptsegnet_amd Warper runs on the HIP engine only; "
                           f"got input on {x.device}")
    if x.dtype != torch.float32:
        raise RuntimeError(f"expected float32 input, got {x.dtype}")
    depth = len(model.encoder_d.down_list) + 1
    if x.shape[2] % (1 << depth) or x.shape[3] % (1 << depth):
        raise ValueError(f"Warper: input {tuple(x.shape[2:])} must be divisible by {1 << depth} in "
                         "both dimensions (the skip connections must match; the reference fails "
                         "otherwise)")
    model._ensure_arena(x.device)
    need_w = any(p.requires_grad for p in model._arena.params)
    grad = torch.is_grad_enabled() and (need_w or x.requires_grad)
    outs = _WarperFn.apply(model._anchors[need_w], x, model, grad)
    return outs[0], list(outs[1:])


class _GridWarpFn(torch.autograd.Function):
    """ResNetMulti.warp on both heads with one warp field (deeplab_multi.py:190-192, 238-255)."""

    @staticmethod
    def forward(ctx, flow, x1, x2):
        ctx.set_materialize_grads(False)
        f = K.nhwc_view(flow)
        if not f.is_contiguous():
            f = f.contiguous()
        a1 = None if x1 is None else K.nhwc_view(x1)
        a2 = K.nhwc_view(x2)
        y1, y2 = K.grid_warp_fwd(f, a1, a2)
        ctx.save = (f, a1, a2)
        return (None if y1 is None else K.as_nchw(y1)), K.as_nchw(y2)

    @staticmethod
    def backward(ctx, gy1, gy2):
        f, a1, a2 = ctx.save
        need_f, need_1, need_2 = ctx.needs_input_grad
        g1 = None if gy1 is None or a1 is None else K.nhwc_view(gy1)
        g2 = None if gy2 is None else K.nhwc_view(gy2)
        if g1 is not None and not g1.is_contiguous():
            g1 = g1.contiguous()
        if g2 is not None and not g2.is_contiguous():
            g2 = g2.contiguous()
        if g1 is None and g2 is None:
            return None, None, None
        dflow, dx1, dx2 = K.grid_warp_bwd(f, a1, a2, g1, g2, need_dflow=need_f, need_dx1=need_1,
                                          need_dx2=need_2)
        ctx.save = None
        return tuple(None if t is None else K.as_nchw(t) for t in (dflow, dx1, dx2))


def grid_warp(flow, x1, x2):
    """(warp(x1, flow), warp(x2, flow)); x1 may be None."""
    if flow.shape[0] != x2.shape[0] or flow.shape[2:] != x2.shape[2:] or (x1 is not None and x1.shape != x2.shape):
        raise ValueError(f"warp: warp field {tuple(flow.shape)} and predictions {tuple(x2.shape)} "
                         "must share N, H, W")
    if flow.shape[1] < 2 or flow.shape[1] % 2:
        raise ValueError("warp: the warp field needs an even number (>= 2) of channels")
    return _GridWarpFn.apply(flow, x1, x2)
