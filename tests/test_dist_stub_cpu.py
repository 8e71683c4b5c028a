"""CPU: the multi-GPU (RCCL) setup and launch order, driven through a stub process group.

No N > 1 RCCL run is possible from the builder's pool (one GPU per box), so the nccl branch's
host logic is pinned here instead (train_gta2cityscapes_multi.py:224-225 is the reference's
DataParallel; ours is one process per GPU with SUM all-reduces of the gradient arenas):

* bench.init_distributed: the local GPU is bound and the ``nccl`` process group is created on
  a HIGH-priority stream with the rank's own device id;
* the trainer's generator buckets: _g_sync_begin installs the hook the engine calls as each
  backward unit's weight gradients are queued; buckets launch in backward order as soon as
  their last unit is done (the first one after layer4.1, long before the stem); the D arenas
  follow; _finish_sync waits every launched collective exactly once, in launch order, and
  nothing is waited before the last launch.
"""
import torch

import bench


class _Opts:
    is_high_priority_stream = False


def test_nccl_init_uses_a_high_priority_stream_on_the_local_gpu(monkeypatch):
    calls = []
    monkeypatch.setattr(bench.dist, "ProcessGroupNCCL", type("PG", (), {"Options": _Opts}))
    bench.init_distributed("nccl", 3, init=lambda *a, **kw: calls.append(("init", a, kw)),
                           set_device=lambda d: calls.append(("set_device", d)))
    assert calls[0] == ("set_device", 3)
    _, args, kw = calls[1]
    assert args == ("nccl",)
    assert kw["device_id"] == torch.device("cuda", 3)
    assert kw["pg_options"].is_high_priority_stream is True
    calls.clear()
    bench.init_distributed("gloo", 1, init=lambda *a, **kw: calls.append(("init", a, kw)),
                           set_device=lambda d: calls.append(("set_device", d)))
    assert calls == [("set_device", 1), ("init", ("gloo",), {})]


class _Work:
    def __init__(self, log, i):
        self.log, self.i = log, i

    def wait(self):
        self.log.append(("wait", self.i))


class _StubDist:
    """torch.distributed stand-in: records every all_reduce (tensor range, op, group)."""

    class ReduceOp:
        SUM = "sum"

    def __init__(self):
        self.log = []
        self.ranges = []

    def all_reduce(self, t, op=None, group=None, async_op=False):
        assert op == "sum" and group == "pg" and async_op
        i = len(self.ranges)
        self.ranges.append((t.data_ptr(), t.numel()))
        self.log.append(("launch", i))
        return _Work(self.log, i)


class _Arena:
    def __init__(self, n):
        self.grad = torch.zeros(n)


def test_bucket_launch_order_and_finish_sync_through_a_stub_process_group(monkeypatch):
    from adaptsegnet_amd import train
    from adaptsegnet_amd.model import DeeplabMulti
    stub = _StubDist()
    monkeypatch.setattr(train, "dist", stub)
    m = DeeplabMulti(num_classes=19)
    m._ensure_arena(torch.device("cpu"))
    tr = train.AdaptSegTrainer.__new__(train.AdaptSegTrainer)
    tr.cfg = train.StepConfig(bucket_mb=32)
    tr.model, tr.pg, tr.world, tr._pending = m, "pg", 8, []
    D1, D2 = type("D", (), {"arena": _Arena(1000)})(), type("D", (), {"arena": _Arena(7)})()
    tr.D1, tr.D2 = D1, D2

    hook = tr._g_sync_begin()
    assert hook is not None and m._grad_hook is hook
    units = m._bwd_units()
    launched_at = {}
    # the engine's done(ordinal) calls of the single-level backward (layer5 gets no gradient)
    for o in range(len(units)):
        if units[o][0] == "layer5":
            continue
        before = len(stub.ranges)
        m._grad_hook(o, None)
        for i in range(before, len(stub.ranges)):
            launched_at[i] = units[o][0]
    tr._g_sync_end(hook)
    assert m._grad_hook is None
    n_g = len(stub.ranges)
    tr._start_sync((tr.D1, tr.D2))
    assert not any(e[0] == "wait" for e in stub.log), "nothing waited before the optimiser"
    tr._finish_sync()
    assert tr._pending == []

    n = len(stub.ranges)
    assert n == n_g + 2
    # every collective waited exactly once, in launch order, after the last launch
    assert stub.log == [("launch", i) for i in range(n)] + [("wait", i) for i in range(n)]
    # generator buckets: backward order, the heads first, the whole arena exactly once
    base = m._arena.grad.data_ptr()
    cover = torch.zeros(m._arena.numel, dtype=torch.int32)
    for ptr, cnt in stub.ranges[:n_g]:
        a = (ptr - base) // 4
        cover[a:a + cnt] += 1
    assert bool((cover == 1).all())
    assert launched_at[0] in ("layer4.1", "layer4.0", "layer6", "layer4.2"), launched_at[0]
    first_stem = min((i for i, u in launched_at.items() if u == "stem"), default=n_g)
    assert first_stem >= 3, "at least three buckets leave before the backward reaches the stem"
    # the discriminators' arenas follow the generator's
    assert stub.ranges[n_g] == (D1.arena.grad.data_ptr(), 1000)
    assert stub.ranges[n_g + 1] == (D2.arena.grad.data_ptr(), 7)


class _LogOpt:
    """SGD / Adam stand-in: LR groups for adjust_learning_rate, a log entry per step."""

    def __init__(self, log, name, groups):
        self.log, self.name = log, name
        self.param_groups = [{"lr": 0.0} for _ in range(groups)]

    def zero_grad(self):
        pass

    def step(self, grad_scale=1.0):
        self.log.append(("step", self.name, grad_scale))


class _GFn(torch.autograd.Function):
    """The generator's autograd Function, reduced to what the data-parallel path sees: its
    backward calls the trainer's hook once per backward unit, as engine._DeeplabMultiFn does
    (done(ordinal) after each unit's weight gradients are queued, done(None) at the end)."""

    @staticmethod
    def forward(ctx, anchor, owner, x):
        ctx.owner = owner
        return anchor * x, anchor * x * 2

    @staticmethod
    def backward(ctx, g1, g2):
        o = ctx.owner
        o.log.append(("bwd", "G"))
        h = o._grad_hook
        if h is not None:
            for k in range(len(o.m._bwd_units())):
                h(k, None)
            h(None, None)
        o.log.append(("bwd_end", "G"))
        return (g1 + 2 * g2).sum().reshape(1), None, None


class _FakeG:
    """DeeplabMulti's arena and bucket plan (the real module, on the CPU) behind a stand-in forward."""

    def __init__(self, log):
        from adaptsegnet_amd.model import DeeplabMulti
        self.log = log
        self.m = DeeplabMulti(num_classes=19)
        self.m._ensure_arena(torch.device("cpu"))
        self.anchor = torch.ones(1, requires_grad=True)
        self._grad_hook = None

    @property
    def arena(self):
        return self.m.arena

    @property
    def _arena(self):
        return self.m._arena

    def _grad_buckets(self, b):
        return self.m._grad_buckets(b)

    def parameters(self):
        return iter([self.anchor])

    def __call__(self, x, size=None):
        return _GFn.apply(self.anchor, self, x)


class _DFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w, owner, x):
        ctx.owner = owner
        return (w * x).sum(dim=1, keepdim=True)

    @staticmethod
    def backward(ctx, g):
        ctx.owner.log.append(("bwd", ctx.owner.name))
        return g.sum().reshape(1), None, None


class _FakeD:
    def __init__(self, log, name, n):
        self.log, self.name = log, name
        self.arena = _Arena(n)
        self.w = torch.ones(1, requires_grad=True)

    def parameters(self):
        return iter([self.w])

    def __call__(self, x):
        return _DFn.apply(self.w, self, x)


def test_multi_level_iter_size_two_launch_order(monkeypatch):
    """The multi-level step (train_gta2cityscapes_multi.py:569-683, the c3 / c5 program) with
    iter_size = 2 at 8 ranks, through a stub process group: the generator's buckets launch only
    from INSIDE the last generator backward of the last sub-iteration (the adversarial one) — not
    from the segmentation backward nor from any backward of sub-iteration 0 — in backward order;
    the D1 / D2 arenas launch after their last backward; every collective is waited once, after
    the last launch and before the first optimiser step; the optimisers scale by 1/world."""
    from adaptsegnet_amd import train
    log = []
    stub = _StubDist()
    stub.log = log
    monkeypatch.setattr(train, "dist", stub)

    class _F:   # functional stand-ins on CPU tensors (the graph is what matters here)
        BCE, MSE = 0, 1
        cross_entropy2d = staticmethod(lambda p, lab, ign=255: p.mean())
        softmax2d = staticmethod(lambda x: x * 1.0)
        adv_loss = staticmethod(lambda d, t, kind: d.mean())
    monkeypatch.setattr(train, "F", _F)

    G = _FakeG(log)
    D1, D2 = _FakeD(log, "D1", 1000), _FakeD(log, "D2", 7)
    tr = train.AdaptSegTrainer.__new__(train.AdaptSegTrainer)
    tr.cfg = train.StepConfig(level="multi-level", gan="LS", iter_size=2, bucket_mb=32,
                              input_size=(8, 4), input_size_target=(8, 4))
    tr.model, tr.D1, tr.D2, tr.warper = G, D1, D2, None
    tr.pg, tr.world, tr._pending, tr._consts, tr.kind = "pg", 8, [], {}, _F.MSE
    tr.opt = _LogOpt(log, "G", 2)
    tr.opt_D1, tr.opt_D2 = _LogOpt(log, "D1", 1), _LogOpt(log, "D2", 1)
    x = torch.randn(1, 3, 4, 8)
    lab = torch.zeros(1, 4, 8, dtype=torch.int64)
    tr._step_body(0, [(x, lab, x), (x, lab, x)])

    g_bwd = [i for i, e in enumerate(log) if e == ("bwd", "G")]
    assert len(g_bwd) == 4   # seg + adversarial, per sub-iteration
    launches = [i for i, e in enumerate(log) if e[0] == "launch"]
    n_buckets = len(G.m._grad_buckets(32 * 2 ** 20))
    g_launch, d_launch = launches[:-2], launches[-2:]
    assert len(g_launch) >= n_buckets
    last_g_end = max(i for i, e in enumerate(log) if e == ("bwd_end", "G"))
    assert all(g_bwd[-1] < i < last_g_end for i in g_launch), "G buckets only inside the last G backward"
    d_bwd = [i for i, e in enumerate(log) if e[0] == "bwd" and e[1] in ("D1", "D2")]
    # per sub-iteration: the adversarial loss back through frozen D1 / D2, then the D steps
    # (D1 + D2 on the source and on the target predictions)
    assert len(d_bwd) == 12
    assert all(i > max(d_bwd) for i in d_launch), "D arenas after their last backward"
    assert stub.ranges[-2] == (D1.arena.grad.data_ptr(), 1000)
    assert stub.ranges[-1] == (D2.arena.grad.data_ptr(), 7)
    waits = [i for i, e in enumerate(log) if e[0] == "wait"]
    steps = [i for i, e in enumerate(log) if e[0] == "step"]
    assert len(waits) == len(launches) and min(waits) > max(launches) and max(waits) < min(steps)
    assert [log[i][1] for i in waits] == list(range(len(launches)))   # launch order
    assert [log[i][1:] for i in steps] == [("G", 1 / 8), ("D1", 1 / 8), ("D2", 1 / 8)]
    # the generator buckets tile the arena once
    base = G.m._arena.grad.data_ptr()
    cover = torch.zeros(G.m._arena.numel, dtype=torch.int32)
    for ptr, cnt in stub.ranges[:-2]:
        cover[(ptr - base) // 4:(ptr - base) // 4 + cnt] += 1
    assert bool((cover == 1).all())
