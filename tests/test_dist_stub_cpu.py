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
