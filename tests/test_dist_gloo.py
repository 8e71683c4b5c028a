"""CPU, world_size 2 (gloo): the data-parallel gradient path of adaptsegnet_amd.train.

The trainer's ``sync_gradients`` SUM-all-reduces each parameter arena's flat gradient
buffer and the optimisers apply ``grad_scale = 1/world``.  Here every rank computes oracle
gradients on ITS shard (per-rank BN statistics, as the reference's per-replica
DataParallel semantics), packs them into a flat buffer exactly like ParamArena does, runs
the trainer's sync, and checks the result equals the mean of both shards' gradients
computed in one process — i.e. the synchronised update equals DataParallel's.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import reference_torch as R


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_grads(rank, layout):
    """Oracle D-step gradients of one shard (small generator layout keeps it fast)."""
    torch.manual_seed(0)
    D = R.to_torch(R.det_state(R.d_specs(), 2002), trainable=lambda k: True)
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.softmax(torch.randn(2, 19, 32, 48, generator=g, dtype=torch.float64), dim=1)
    loss = R.adv_loss(R.d_forward(D, x), rank % 2, "Vanilla")
    loss.backward()
    return torch.cat([D[k].grad.flatten() for k in D])


class _FakeArena:
    def __init__(self, grad):
        self.grad = grad


class _FakeModel:
    def __init__(self, grad):
        self.arena = _FakeArena(grad)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from adaptsegnet_amd.train import AdaptSegTrainer
        grad = _shard_grads(rank, None).clone()
        tr = AdaptSegTrainer.__new__(AdaptSegTrainer)   # sync only: no GPU models needed
        tr.model, tr.D1, tr.D2, tr.pg = _FakeModel(grad), None, None, None
        tr.world = dist.get_world_size()
        tr.sync_gradients()
        out[rank] = (grad / tr.world).clone()          # what the optimiser sees (grad_scale)
    finally:
        dist.destroy_process_group()


def _overlap_worker(rank, world, port, out):
    """The step's overlapped order: G's all-reduce launched asynchronously, more work (the
    D passes) queued while it runs, then the D arenas, then one wait for all of them."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from adaptsegnet_amd.train import AdaptSegTrainer
        g = _shard_grads(rank, None).clone()
        d1 = torch.full((1000,), float(rank + 1), dtype=torch.float64)
        d2 = torch.arange(7, dtype=torch.float64) * (rank + 1)
        tr = AdaptSegTrainer.__new__(AdaptSegTrainer)
        tr.model, tr.D1, tr.D2, tr.pg = _FakeModel(g), _FakeModel(d1), _FakeModel(d2), None
        tr.world = dist.get_world_size()
        tr._start_sync((tr.model,))
        busy = _shard_grads(1 - rank, None)          # the D passes of the step
        tr._start_sync((tr.D1, tr.D2))
        tr._finish_sync()
        out[rank] = (g.clone(), d1.clone(), d2.clone(), float(busy.sum()))
    finally:
        dist.destroy_process_group()


def test_overlapped_sync_matches_blocking_sync():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_overlap_worker, args=(world, port, out), nprocs=world, join=True)
    g_sum = _shard_grads(0, None) + _shard_grads(1, None)
    for r in range(world):
        g, d1, d2, _ = out[r]
        assert torch.allclose(g, g_sum, rtol=1e-12, atol=1e-15)
        assert torch.equal(d1, torch.full((1000,), 3.0, dtype=torch.float64))
        assert torch.equal(d2, torch.arange(7, dtype=torch.float64) * 3)
    assert torch.equal(out[0][0], out[1][0])


def test_gradient_sync_matches_dataparallel_mean():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    expected = (_shard_grads(0, None) + _shard_grads(1, None)) / 2
    for r in range(world):
        assert torch.allclose(out[r], expected, rtol=1e-12, atol=1e-15)
    assert torch.equal(out[0], out[1])  # every rank applies the identical update


def test_sgd_grad_scale_folds_the_average():
    """SGD with grad_scale=1/world on the summed gradient == SGD on the averaged gradient
    (the fused kernel applies g*scale before weight decay, as the oracle-pinned math)."""
    import warnings
    p0 = torch.randn(64, dtype=torch.float64)
    g_sum = torch.randn(64, dtype=torch.float64)
    world = 4
    ref = torch.nn.Parameter(p0.clone())
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        opt = torch.optim.SGD([ref], lr=0.1, momentum=0.9, weight_decay=5e-4, foreach=False)
    ref.grad = g_sum / world
    opt.step()
    # restatement of adaptseg_sgd_step (first step, multiplicity 1) with grad_scale
    d = g_sum * (1.0 / world) + 5e-4 * p0
    assert torch.allclose(ref.detach(), p0 - 0.1 * d, rtol=1e-12)


# ---------------------------------------------------------------------------------------
# Bucketed generator all-reduce (train._BucketAllReduce + DeeplabMulti._grad_buckets)
# ---------------------------------------------------------------------------------------

def _cpu_deeplab():
    from adaptsegnet_amd.model import DeeplabMulti
    m = DeeplabMulti(num_classes=19)
    m._ensure_arena(torch.device("cpu"))
    return m


@pytest.mark.parametrize("mb", [8, 32, 1000])
def test_grad_buckets_tile_the_arena_in_backward_order(mb):
    m = _cpu_deeplab()
    A = m._arena
    buckets = m._grad_buckets(mb * 2 ** 20)
    units = m._bwd_units()
    ords = [o for o, _ in buckets]
    assert ords == sorted(ords) and ords[-1] == len(units) - 1
    cover = torch.zeros(A.numel, dtype=torch.int32)
    for _, runs in buckets:
        for a, b in runs:
            assert 0 <= a < b <= A.numel
            cover[a:b] += 1
    assert bool((cover == 1).all()), "every arena element in exactly one bucket"
    # the first bucket holds the heads: layer6 and layer4 finish first in backward
    first = {A.params[i] for i in range(len(A.params))
             if any(a <= A.offsets[i] < b for a, b in buckets[0][1])}
    assert all(p in first for p in m.layer6.parameters())
    if mb == 1000:
        assert len(buckets) == 1
    else:
        sizes = [4 * sum(b - a for a, b in runs) for _, runs in buckets]
        assert all(s >= mb * 2 ** 20 for s in sizes[:-1])
        assert len(buckets) >= 2 and all(s < 3 * mb * 2 ** 20 + 24 * 2 ** 20 for s in sizes)


def _bucket_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from adaptsegnet_amd.train import _BucketAllReduce
        m = _cpu_deeplab()
        g = torch.Generator().manual_seed(7 + rank)
        grad = torch.randn(m._arena.numel, generator=g, dtype=torch.float32)
        orig = grad.clone()
        tr = type("T", (), {})()
        tr._pending, tr.pg = [], None
        hook = _BucketAllReduce(tr, grad, m._grad_buckets(16 * 2 ** 20))
        # the single-level backward skips layer5 (ordinal len(layer4) + 1) and the stem unit
        skip = {len(m.layer4) + 1, len(m._bwd_units()) - 1}
        for o in range(len(m._bwd_units())):
            if o not in skip:
                hook(o, None)
        hook(None, None)
        for w in tr._pending:
            w.wait()
        out[rank] = (orig, grad.clone(), list(hook.launched))
    finally:
        dist.destroy_process_group()


def test_bucketed_allreduce_sums_every_element_once():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_worker, args=(world, port, out), nprocs=world, join=True)
    total = out[0][0] + out[1][0]
    for r in range(world):
        assert torch.allclose(out[r][1], total, rtol=1e-6, atol=1e-6)
    assert torch.equal(out[0][1], out[1][1])
    launched = out[0][2]
    assert len(launched) > 3 and launched == out[1][2]
