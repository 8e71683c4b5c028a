"""The AdaptSegNet adversarial training step on the HIP engine (single- and multi-level).

Restates the per-iteration body of /root/reference/train_gta2cityscapes_multi.py:
  single-level  :379-464  (G: seg loss on source, adversarial loss on target through the
                            frozen D2; D2: source -> 0, target -> 1, each loss / 2)
  multi-level   :570-683  (two heads, two discriminators, loss_seg2 + lambda_seg*loss_seg1)
  poly LR       :162-177,  SGD(momentum .9, wd 5e-4) + Adam(.9, .99)  :532-540
Resolved reference gaps:
  * the multi-level call ``model(images)`` (:597,615) lacks ``input_size`` and raises in the
    reference; here source predictions are upsampled to ``input_size`` and target ones to
    ``input_size_target`` (``target_size='target'``), or to the source size as the fork's
    single-level branch does (:421, ``target_size='source'``, the single-level default);
  * ``SOURCE_ONLY = True`` (:24) is not hard-wired: ``StepConfig.level`` selects the
    adversarial steps or ``"source-only"`` (:259-286, segmentation loss only);
  * the fork's warper (:217-220, 271-275, 401-405) is applied when a ``Warper`` is given: its
    field warps the source predictions (source-only and single-level).  The reference's
    single-level branch reuses the source field for the target prediction (:421) and then
    crashes in the target backward (the field's graph was freed by the source backward); here
    the target is warped by the same field, detached.  The warper's parameters are in no
    optimiser (:244,347,532), so their gradients only accumulate, as in the reference.
Differences that do not change results: loss scalings (``lambda * loss / iter_size``) are
passed as the initial gradient of ``backward`` instead of multiplying the loss tensors, the
constant label tensors (:621, ...) are folded into the loss kernels, and the per-loss
``.item()`` host syncs are deferred to ``StepLosses.values()``.

Data parallel (one process per GPU): every rank runs the step on its own shard, and SUM
all-reduces of the gradient arenas replace DataParallel's gradient gather
(train_gta2cityscapes_multi.py:224-225); the 1/world average is folded into the optimiser.
DeeplabMulti's 178 MB arena is reduced in buckets (``bucket_mb``) launched from inside the
step's last generator backward as each bucket's weight gradients are queued (layer6 and layer4
first), so the collectives overlap the rest of that backward; the discriminators' arenas follow
their last backward.  BN statistics stay per-rank, as in the reference's per-replica
DataParallel semantics.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from . import engine
from . import functional as F
from . import kernels as K
from .optim import SGD, Adam, lr_poly


@dataclass
class StepConfig:
    level: str = "single-level"          # or "multi-level", "source-only"
    gan: str = "Vanilla"                 # "Vanilla" (BCEWithLogits) or "LS" (MSE)
    num_classes: int = 19
    input_size: tuple = (1024, 512)      # (W, H) of source images
    input_size_target: tuple = (1024, 512)
    target_size: str = "auto"            # "source" | "target" | "auto" (single: source, multi: target)
    iter_size: int = 1
    learning_rate: float = 2.5e-4
    learning_rate_D: float = 1e-4
    momentum: float = 0.9
    weight_decay: float = 5e-4
    power: float = 0.9
    num_steps: int = 250000
    lambda_seg: float = 0.1
    lambda_adv_target1: float = 0.0002
    lambda_adv_target2: float = 0.001
    ignore_label: int = 255
    # run the target-domain generator forward (+ its D forward) on a second HIP stream while
    # the source-domain backward executes (independent: same weights, read-only, separate
    # gradient kernels); the target backward then waits for the source backward.  Results are
    # bit-identical to the sequential order (tests/test_model_gpu.py).  "auto" (the default):
    # on for DeeplabMulti — the backward alone does not fill the chip, the forward beside it
    # does: c2 +1.3 %, c3 +1.1 %, c5 +3.6 % (profiles/r5/overlap_ab.txt) — off for DeeplabVGG
    # (c4 -0.6 %).
    overlap_domains: bool | str = "auto"
    # with overlap_domains: enqueue the target forward BEFORE the source backward, so its kernels
    # are in the side stream's queue when the backward starts instead of after the host has
    # issued the whole backward (≈1,000 launches); same kernels, same inputs, bit-identical.
    # Off: within ±0.6 % at c2 / c3 / c5 (profiles/r5/target_first_ab.txt) — the host already
    # runs far enough ahead of the GPU
    target_first: bool = False
    # run the discriminator step (its forwards on the detached predictions and its backwards,
    # train:435-461 / 642-679) on its own HIP stream as soon as the target forward is done, beside
    # the step's last generator backward: it reads only the detached predictions and D's weights
    # (unchanged until the optimisers), and writes only D's gradient arena, which that backward
    # does not touch (D's parameters are frozen while its graph is built).  Results are
    # bit-identical to the sequential order (tests/test_model_gpu.py).
    overlap_d: bool = False
    # D's own step on the target prediction reuses the forward the generator's adversarial loss
    # ran (same input, same weights: bit-identical, engine.DiscForward) instead of running D and
    # its softmax again — one D forward per discriminator and step fewer
    d_reuse: bool = True
    # single-level: DeeplabMulti computes only the head the step uses (the reference's
    # ``_, pred2 = model(...)`` discards layer5's; ResNetMulti.forward(first_head=False))
    second_head_only: bool = True
    # data parallel: size of the generator's gradient all-reduce buckets (DeeplabMulti); 0 =
    # one all-reduce of the whole arena after its last backward
    bucket_mb: float = 32.0
    # HIP stream priority of the step's main chain (None: the caller's stream; "auto": high
    # for DeeplabMulti, the caller's stream for DeeplabVGG); see step()
    main_priority: int | str | None = "auto"


@dataclass
class StepLosses:
    tensors: dict = field(default_factory=dict)

    def add(self, name, t, scale):
        self.tensors.setdefault(name, []).append((t, scale))

    def values(self) -> dict:
        """Host values (one device sync), summed like the reference's *_value accumulators."""
        return {k: sum(float(t.detach()) * s for t, s in v) for k, v in self.tensors.items()}


class AdaptSegTrainer:
    """Owns the optimisers and runs one adversarial iteration per ``step()`` call."""

    def __init__(self, model, model_D1, model_D2, cfg: StepConfig, process_group=None, warper=None):
        self.model, self.D1, self.D2, self.cfg = model, model_D1, model_D2, cfg
        self.warper = warper
        if cfg.level not in ("single-level", "multi-level", "source-only"):
            raise ValueError(f"unknown level {cfg.level!r}")
        if cfg.level == "multi-level" and model_D1 is None:
            raise ValueError("multi-level needs model_D1")
        if cfg.level == "multi-level" and getattr(model, "single_output", False):
            raise ValueError("multi-level needs a two-head generator (DeeplabMulti)")
        if cfg.level != "source-only" and model_D2 is None:
            raise ValueError(f"{cfg.level} needs model_D2")
        if warper is not None and (cfg.level == "multi-level" or getattr(model, "single_output", False)):
            raise ValueError("the warper applies to DeeplabMulti's source-only and single-level steps "
                             "(train_gta2cityscapes_multi.py:271-275, 401-405)")
        self.opt = SGD(model, cfg.learning_rate, cfg.momentum, cfg.weight_decay)
        self.opt_D1 = Adam(model_D1, cfg.learning_rate_D, betas=(0.9, 0.99)) if model_D1 is not None else None
        self.opt_D2 = Adam(model_D2, cfg.learning_rate_D, betas=(0.9, 0.99)) if model_D2 is not None else None
        self.kind = F.BCE if cfg.gan == "Vanilla" else F.MSE
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        self._consts = {}
        self._pending = []

    # -- helpers -------------------------------------------------------------------------
    def _c(self, v: float, device):
        key = (float(v), device)
        t = self._consts.get(key)
        if t is None:
            t = self._consts[key] = torch.full((), float(v), dtype=torch.float32, device=device)
        return t

    # -- stream overlap of the two domains -----------------------------------------------------
    _streams: dict = {}

    def _overlap_domains(self) -> bool:
        ov = self.cfg.overlap_domains
        if ov == "auto":
            return not getattr(self.model, "single_output", False)
        return bool(ov)

    def _overlap_begin(self, device):
        """After the source forward: returns (main, side, event) or None (overlap off / CPU)."""
        if not self._overlap_domains() or device.type != "cuda":
            return None
        side = AdaptSegTrainer._streams.get(device.index)
        if side is None:
            side = AdaptSegTrainer._streams[device.index] = torch.cuda.Stream(device)
        main = torch.cuda.current_stream(device)
        ev = torch.cuda.Event()
        ev.record(main)   # the target pass starts after the source forward (BN running stats)
        return main, side, ev

    def _target_ctx(self, ov):
        if ov is None:
            return contextlib.nullcontext()
        main, side, ev = ov
        side.wait_event(ev)
        return torch.cuda.stream(side)

    @staticmethod
    def _join_source(ov):
        """Before the target-domain G backward: the source backward (main stream) must have
        finished writing the gradient arena it accumulates into."""
        if ov is not None:
            ov[1].wait_stream(ov[0])

    _d_streams: dict = {}

    def _d_fork(self, device):
        """After the target forward (+ its D forward), on the stream that ran it: an event the
        discriminator step's stream waits on, or None (overlap_d off / CPU)."""
        if not self.cfg.overlap_d or device.type != "cuda":
            return None
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        return ev

    def _d_ctx(self, ev, device, *tensors):
        """The discriminator step's stream context: waits for ``ev`` only; ``tensors`` (made on
        other streams) are marked used on it.  The main stream joins it before the optimisers."""
        if ev is None:
            return contextlib.nullcontext()
        ds = AdaptSegTrainer._d_streams.get(device.index)
        if ds is None:
            ds = AdaptSegTrainer._d_streams[device.index] = torch.cuda.Stream(device)
        ds.wait_event(ev)
        for t in tensors:
            t.record_stream(ds)
        self.__dict__.setdefault("_d_used", set()).add(device.index)
        return torch.cuda.stream(ds)

    def _d_join(self, device):
        if device.index in self.__dict__.get("_d_used", ()):
            torch.cuda.current_stream(device).wait_stream(AdaptSegTrainer._d_streams[device.index])
            self._d_used.discard(device.index)

    @staticmethod
    def _overlap_end(ov, *tensors):
        if ov is None:
            return
        main, side, _ = ov
        main.wait_stream(side)
        for t in tensors:
            t.record_stream(main)   # produced on the side stream, read on the main stream

    def _d_keep(self, D):
        """A DiscForward to keep D's target forward in (d_reuse, HIP-engine discriminators)."""
        return engine.DiscForward() if self.cfg.d_reuse and hasattr(D, "_convs") else None

    @staticmethod
    def _d_out(D, x, keep):
        return D(x) if keep is None else engine.discriminator_forward(D, x, keep=keep)

    @staticmethod
    def _d_again(D, pred, keep):
        """D on the detached target prediction for D's own step: the kept forward when there is one."""
        return D(F.softmax2d(pred)) if keep is None else engine.discriminator_replay(D, keep)

    @staticmethod
    def _kept(*keeps):
        return [t for k in keeps if k is not None for t in k.tensors()]

    def _backward(self, losses, scales):
        dev = losses[0].device
        torch.autograd.backward(list(losses), grad_tensors=[self._c(s, dev) for s in scales])

    @staticmethod
    def _set_requires_grad(model, flag):
        for p in model.parameters():
            p.requires_grad = flag

    def adjust_learning_rate(self, i_iter):
        c = self.cfg
        lr = lr_poly(c.learning_rate, i_iter, c.num_steps, c.power)
        self.opt.param_groups[0]["lr"] = lr
        self.opt.param_groups[1]["lr"] = lr * 10
        lr_d = lr_poly(c.learning_rate_D, i_iter, c.num_steps, c.power)
        for o in (self.opt_D1, self.opt_D2):
            if o is not None:
                o.param_groups[0]["lr"] = lr_d

    def _target_size(self):
        c = self.cfg
        mode = c.target_size
        if mode == "auto":
            mode = "source" if c.level == "single-level" else "target"
        return c.input_size if mode == "source" else c.input_size_target

    def sync_gradients(self):
        """SUM all-reduce of each parameter arena's gradients (RCCL on ROCm), blocking."""
        self._start_sync((self.model, self.D1, self.D2))
        self._finish_sync()

    def _start_sync(self, models):
        """Launch the arena all-reduces of ``models`` asynchronously.  RCCL orders them after
        the work already queued on the current stream (the gradients they read) and runs them
        on its own stream, so they overlap whatever the step launches next."""
        if self.world == 1:
            return
        pending = self.__dict__.setdefault("_pending", [])
        for m in models:
            if m is not None and m.arena is not None:
                pending.append(dist.all_reduce(m.arena.grad, op=dist.ReduceOp.SUM,
                                                     group=self.pg, async_op=True))

    def _g_sync_begin(self):
        """Before the step's last generator backward: install the bucketed all-reduce hook on
        a generator that supports it (DeeplabMulti).  Returns the hook or None."""
        if self.world == 1 or self.cfg.bucket_mb <= 0 or not hasattr(self.model, "_grad_buckets"):
            return None
        if getattr(self.model, "_arena", None) is None:
            return None
        hook = _BucketAllReduce(self, self.model.arena.grad,
                                self.model._grad_buckets(int(self.cfg.bucket_mb * 2 ** 20)))
        self.model._grad_hook = hook
        return hook

    def _g_sync_end(self, hook):
        """After the step's last generator backward: every bucket (or the whole arena) has its
        all-reduce in flight."""
        if hook is None:
            self._start_sync((self.model,))
            return
        self.model._grad_hook = None
        hook(None, None)
        self.g_allreduce_ranges = list(hook.launched)   # (start, end) arena ranges, launch order

    def _finish_sync(self):
        """Make the current stream wait for every launched all-reduce (no host sync)."""
        for w in self.__dict__.get("_pending", ()):
            w.wait()
        self._pending = []

    # -- the step --------------------------------------------------------------------------
    _hp_streams: dict = {}

    def step(self, i_iter, batches):
        """One iteration.  The step's main chain (forwards, data gradients, BN, losses,
        optimisers) runs on a HIP stream of priority ``cfg.main_priority`` (-1, high, for
        DeeplabMulti), so the hardware scheduler favours it over the weight-gradient side stream
        that fills the gaps the HBM-bound BN passes leave: +0.9 % c2, +0.2 % c3, ±0 c5, but
        -1.7 % for DeeplabVGG (c4: no BN, so it runs on the caller's stream).  The caller's
        stream waits for it at the end.  ``main_priority=None`` runs on the caller's stream."""
        prio = self.cfg.main_priority
        if prio == "auto":   # VGG has no BN passes for the side stream to fill: -1.7 % with it
            prio = None if getattr(self.model, "single_output", False) else -1
        dev = next(self.model.parameters()).device
        # each conv's weight pack is built once per step (the optimisers, the only writers of the
        # weights, run after the step's last conv): kernels.weight_pack_scope
        if prio is None or dev.type != "cuda":
            with K.weight_pack_scope():
                return self._step_body(i_iter, batches)
        batches = list(batches)
        key = (dev.index, prio)
        hp = AdaptSegTrainer._hp_streams.get(key)
        if hp is None:
            hp = AdaptSegTrainer._hp_streams[key] = torch.cuda.Stream(dev, priority=prio)
        cur = torch.cuda.current_stream(dev)
        hp.wait_stream(cur)
        with torch.cuda.stream(hp), K.weight_pack_scope():
            L = self._step_body(i_iter, batches)
        cur.wait_stream(hp)
        return L

    def _step_body(self, i_iter, batches):
        """batches: iterable of ``iter_size`` tuples (images, labels, images_target).

        Multi-GPU: the generator's gradients are final after its adversarial backward of the
        last sub-iteration, so their all-reduce (the 178 MB arena) is launched right there and
        overlaps the discriminator forward/backward passes; the discriminators' (11 MB each)
        follow their last backward.  The optimisers wait for both."""
        c = self.cfg
        L = StepLosses()
        self.opt.zero_grad()
        for o in (self.opt_D1, self.opt_D2):
            if o is not None:
                o.zero_grad()
        self.adjust_learning_rate(i_iter)
        inv = 1.0 / c.iter_size
        tsize = self._target_size()
        batches = list(batches)
        self._pending = []
        for idx, batch in enumerate(batches):
            g_done = _GSync(self) if idx == len(batches) - 1 else None
            if c.level == "source-only":
                self._sub_source_only(batch[0], batch[1], inv, L, g_done)
                continue
            images, labels, images_t = batch
            if c.level == "single-level":
                self._sub_single(images, labels, images_t, inv, tsize, L, g_done)
            else:
                self._sub_multi(images, labels, images_t, inv, tsize, L, g_done)
        if not batches:
            self._start_sync((self.model,))
        if batches and c.level != "source-only":
            self._d_join(next(self.model.parameters()).device)
        self._start_sync((self.D1, self.D2))
        self._finish_sync()
        gs = 1.0 / self.world
        self.opt.step(grad_scale=gs)
        for o in (self.opt_D1, self.opt_D2):
            if o is not None:
                o.step(grad_scale=gs)
        return L

    def _pred_single(self, images, size, flow=None):
        """The single-level prediction at ``size`` = (W, H): DeeplabMulti's second head (warped
        by ``flow`` when given), or a single-map model (DeeplabVGG, config c4) followed by the
        caller-side ``interp``."""
        if getattr(self.model, "single_output", False):
            return F.interp(self.model(images), (size[1], size[0]))
        if self.cfg.second_head_only and getattr(self.model, "second_head_only_ok", False):
            return self.model(images, size, flow, first_head=False)[1]
        return self.model(images, size, flow)[1]

    def _flow(self, images):
        return None if self.warper is None else self.warper(images)[0]

    def _sub_source_only(self, images, labels, inv, L, g_done=None):
        """train_gta2cityscapes_multi.py:259-286: warper (if any), segmentation loss on the
        second head, backward; the step is the generator's SGD only."""
        pred2 = self._pred_single(images, self.cfg.input_size, self._flow(images))
        loss_seg2 = F.cross_entropy2d(pred2, labels, self.cfg.ignore_label)
        if g_done is not None:
            g_done.begin()
        self._backward([loss_seg2], [inv])
        L.add("loss_seg2", loss_seg2, inv)
        if g_done is not None:
            g_done.end()

    def _sub_single(self, images, labels, images_t, inv, tsize, L, g_done=None):
        """train_gta2cityscapes_multi.py:385-461."""
        c, D2 = self.cfg, self.D2
        self._set_requires_grad(D2, False)
        flow = self._flow(images)
        pred2 = self._pred_single(images, c.input_size, flow)
        loss_seg2 = F.cross_entropy2d(pred2, labels, c.ignore_label)
        ov = self._overlap_begin(pred2.device)
        keep2 = self._d_keep(D2)

        def target_forward():
            with self._target_ctx(ov):
                pt2 = self._pred_single(images_t, tsize, None if flow is None else flow.detach())
                return pt2, F.adv_loss(self._d_out(D2, F.softmax2d(pt2), keep2), 0.0, self.kind)

        first = ov is not None and c.target_first
        if first:
            pred_target2, loss_adv_target2 = target_forward()
        self._backward([loss_seg2], [inv])
        L.add("loss_seg2", loss_seg2, inv)
        if not first:
            pred_target2, loss_adv_target2 = target_forward()

        with self._target_ctx(ov):
            dev_ = loss_adv_target2.device
            dfork = self._d_fork(dev_)
            self._join_source(ov)
            if g_done is not None:
                g_done.begin()
            self._backward([loss_adv_target2], [c.lambda_adv_target2 * inv])
            L.add("loss_adv_target2", loss_adv_target2, inv)
            if g_done is not None:
                g_done.end()
        self._overlap_end(ov, pred_target2, loss_adv_target2, *self._kept(keep2))

        self._set_requires_grad(D2, True)
        pred2 = pred2.detach()
        pred_target2 = pred_target2.detach()
        with self._d_ctx(dfork, dev_, pred2, pred_target2, *self._kept(keep2)):
            loss_d2 = F.adv_loss(D2(F.softmax2d(pred2)), 0.0, self.kind)
            self._backward([loss_d2], [inv / 2])
            L.add("loss_D2", loss_d2, inv / 2)
            loss_d2 = F.adv_loss(self._d_again(D2, pred_target2, keep2), 1.0, self.kind)
            self._backward([loss_d2], [inv / 2])
            L.add("loss_D2", loss_d2, inv / 2)

    def _sub_multi(self, images, labels, images_t, inv, tsize, L, g_done=None):
        """train_gta2cityscapes_multi.py:578-679."""
        c, D1, D2 = self.cfg, self.D1, self.D2
        self._set_requires_grad(D1, False)
        self._set_requires_grad(D2, False)
        pred1, pred2 = self.model(images, c.input_size)
        loss_seg1 = F.cross_entropy2d(pred1, labels, c.ignore_label)
        loss_seg2 = F.cross_entropy2d(pred2, labels, c.ignore_label)
        ov = self._overlap_begin(pred2.device)
        keep1, keep2 = self._d_keep(D1), self._d_keep(D2)

        def target_forward():
            with self._target_ctx(ov):
                pt1, pt2 = self.model(images_t, tsize)
                return (pt1, pt2, F.adv_loss(self._d_out(D1, F.softmax2d(pt1), keep1), 0.0, self.kind),
                        F.adv_loss(self._d_out(D2, F.softmax2d(pt2), keep2), 0.0, self.kind))

        first = ov is not None and c.target_first
        if first:
            pred_target1, pred_target2, loss_adv1, loss_adv2 = target_forward()
        self._backward([loss_seg2, loss_seg1], [inv, c.lambda_seg * inv])
        L.add("loss_seg1", loss_seg1, inv)
        L.add("loss_seg2", loss_seg2, inv)
        if not first:
            pred_target1, pred_target2, loss_adv1, loss_adv2 = target_forward()

        with self._target_ctx(ov):
            dev_ = loss_adv2.device
            dfork = self._d_fork(dev_)
            self._join_source(ov)
            if g_done is not None:
                g_done.begin()
            self._backward([loss_adv1, loss_adv2],
                           [c.lambda_adv_target1 * inv, c.lambda_adv_target2 * inv])
            L.add("loss_adv_target1", loss_adv1, inv)
            L.add("loss_adv_target2", loss_adv2, inv)
            if g_done is not None:
                g_done.end()
        self._overlap_end(ov, pred_target1, pred_target2, loss_adv1, loss_adv2, *self._kept(keep1, keep2))

        self._set_requires_grad(D1, True)
        self._set_requires_grad(D2, True)
        pred1, pred2 = pred1.detach(), pred2.detach()
        pred_target1, pred_target2 = pred_target1.detach(), pred_target2.detach()
        with self._d_ctx(dfork, dev_, pred1, pred2, pred_target1, pred_target2, *self._kept(keep1, keep2)):
            loss_d1 = F.adv_loss(D1(F.softmax2d(pred1)), 0.0, self.kind)
            loss_d2 = F.adv_loss(D2(F.softmax2d(pred2)), 0.0, self.kind)
            self._backward([loss_d1], [inv / 2])
            self._backward([loss_d2], [inv / 2])
            L.add("loss_D1", loss_d1, inv / 2)
            L.add("loss_D2", loss_d2, inv / 2)
            loss_d1 = F.adv_loss(self._d_again(D1, pred_target1, keep1), 1.0, self.kind)
            loss_d2 = F.adv_loss(self._d_again(D2, pred_target2, keep2), 1.0, self.kind)
            self._backward([loss_d1], [inv / 2])
            self._backward([loss_d2], [inv / 2])
            L.add("loss_D1", loss_d1, inv / 2)
            L.add("loss_D2", loss_d2, inv / 2)


class _GSync:
    """begin() / end() around the step's last generator backward (the gradients are final
    after it): bucketed all-reduces launched from inside that backward, or one whole-arena
    all-reduce after it."""

    def __init__(self, trainer):
        self.tr, self.hook = trainer, None

    def begin(self):
        self.hook = self.tr._g_sync_begin()

    def end(self):
        self.tr._g_sync_end(self.hook)


class _BucketAllReduce:
    """The generator backward's data-parallel hook (DeeplabMulti._grad_hook).

    ``buckets`` = DeeplabMulti._grad_buckets(): [(last_unit_ordinal, [(start, end), ...])] in
    completion order.  hook(ordinal, stream) launches the SUM all-reduce of every bucket whose
    last backward unit is <= ordinal (units skipped by this backward, e.g. layer5 in the
    single-level step, ride with the next unit); hook(None, _) launches the rest.  The
    collectives are issued with ``stream`` (the weight-gradient side stream) current, so the
    process group orders them after the weight-gradient GEMMs already queued there and they run
    while the backward continues; the optimiser's stream waits for them in _finish_sync."""

    def __init__(self, trainer, grad, buckets):
        self.tr, self.grad, self.buckets, self.next = trainer, grad, buckets, 0
        self.launched = []           # (start, end) ranges, in launch order (tests)

    def __call__(self, ordinal, stream):
        while self.next < len(self.buckets) and (ordinal is None or self.buckets[self.next][0] <= ordinal):
            ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
            with ctx:
                for a, b in self.buckets[self.next][1]:
                    self.tr._pending.append(dist.all_reduce(self.grad[a:b], op=dist.ReduceOp.SUM,
                                                            group=self.tr.pg, async_op=True))
                    self.launched.append((a, b))
            self.next += 1
