"""Two data-parallel ranks of the real adversarial step on ONE GPU (gloo process group).

SURVEY.md §8(e) semantics: each rank runs AdaptSegTrainer.step on its own shard with real
DeeplabMulti / FCDiscriminator models; the generator's gradient arena is SUM-all-reduced in
buckets launched from inside its last backward (train._BucketAllReduce), the
discriminators' after their last backward, and the optimisers apply 1/world.  The result
must equal the fp64 oracle's step with the mean of the per-shard gradients — which is the
oracle's iter_size = 2 step over [shard 0, shard 1] (train:569-683: each sub-batch's losses
scaled by 1/2, gradients accumulated, per-sub-batch BN statistics; eval-mode BN here, the
well-conditioned check, as tests/test_model_gpu.py::test_iter_size_two_accumulates_sub_batches).

Tolerances (as that test): per-rank-mean losses within 1e-4 rel of the fp64 oracle; the
generator's per-group parameter update within 2x the fp32 oracle's own distance to fp64
+ 1e-4; both ranks' parameters bit-identical after every step.  The gloo backend stands in
for RCCL (one GPU on the test box); the collective placement and arithmetic are the same
code path as with backend "nccl".
"""
import os
import socket
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import reference_torch as R

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = [("single-level", "Vanilla"), ("multi-level", "Vanilla")]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shards():
    shapes = ((2, 3, 41, 57), (2, 41, 57), (2, 3, 33, 49))
    return [(torch.from_numpy(R.det_images(shapes[0], 11 + 20 * r)),
             torch.from_numpy(R.det_labels(shapes[1], 12 + 20 * r)),
             torch.from_numpy(R.det_images(shapes[2], 13 + 20 * r))) for r in range(2)]


def _rank(rank, world, port, level, gan, iters, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import test_model_gpu as T
        from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
        torch.cuda.set_device(0)
        m, d1, d2 = T.build_g(), T.build_d(2001), T.build_d(2002)
        m.eval()
        cfg = dict(level=level, gan=gan, input_size=(57, 41), input_size_target=(49, 33))
        tr = AdaptSegTrainer(m, d1 if level == "multi-level" else None, d2,
                             StepConfig(**cfg, bucket_mb=4.0))
        xs, lab, xt = _shards()[rank]
        batch = [(xs.float().to(DEV), lab.to(DEV), xt.float().to(DEV))]
        losses = [tr.step(it, batch).values() for it in range(iters)]
        torch.cuda.synchronize()
        torch.save({"losses": losses, "G": {k: v.detach().cpu() for k, v in m.state_dict().items()},
                    "D2": {k: v.detach().cpu() for k, v in d2.state_dict().items()},
                    "D1": {k: v.detach().cpu() for k, v in d1.state_dict().items()},
                    "ranges": tr.g_allreduce_ranges},
                   os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("level,gan", CASES)
def test_two_rank_step_equals_mean_of_shard_gradients(level, gan):
    import test_model_gpu as T
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    iters, world = 2, 2
    with tempfile.TemporaryDirectory() as outdir:
        mp.spawn(_rank, args=(world, _free_port(), level, gan, iters, outdir), nprocs=world, join=True)
        res = [torch.load(os.path.join(outdir, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    cfg = dict(level=level, gan=gan, input_size=(57, 41), input_size_target=(49, 33), iter_size=2)
    subs = _shards()

    def oracle(dtype):
        G = R.to_torch(R.det_state(R.g_specs(), 1338), dtype=dtype, trainable=R.g_trainable)
        D1 = R.to_torch(R.det_state(R.d_specs(), 2001), dtype=dtype, trainable=lambda k: True)
        D2 = R.to_torch(R.det_state(R.d_specs(), 2002), dtype=dtype, trainable=lambda k: True)
        opts = R.make_optimizers(G, D1 if level == "multi-level" else None, D2, R.DEFAULT_CFG | cfg)
        b = [(a.to(dtype), l, t.to(dtype)) for a, l, t in subs]
        return G, D2, [R.oracle_step(G, D1, D2, opts, cfg, it, b, bn_train=False) for it in range(iters)]

    G, D2, ref = oracle(torch.float64)
    G32, D232, _ = oracle(torch.float32)
    # the generator's all-reduce went out in several buckets, heads first
    ranges = res[0]["ranges"]
    assert len(ranges) > 3, ranges
    # every rank applies the identical update
    for name in ("G", "D1", "D2"):
        for k, v in res[0][name].items():
            assert torch.equal(v, res[1][name][k]), (name, k)
    for it in range(iters):
        for k, v in ref[it].items():
            got = sum(r["losses"][it][k] for r in res) / world
            print(f"dp2 iter{it} {k}: mean over ranks={got:.7f} fp64 oracle={v:.7f}")
            assert abs(got - v) <= 1e-4 * abs(v) + 1e-7, (it, k, got, v)
    g0 = R.det_state(R.g_specs(), 1338)
    for gname, keys in T._groups(G, level).items():
        dref = T._updates(G, keys, g0)
        f, c = T.frob(T._updates(None, keys, g0, res[0]["G"]), dref)
        f32, _ = T.frob(T._updates(G32, keys, g0), dref)
        print(f"dp2 {gname} update: rel-frob {f:.3e} (fp32 oracle {f32:.3e}) cos {c:.8f}")
        assert f <= 2 * f32 + 1e-4, (gname, f, f32)
    d0 = R.det_state(R.d_specs(), 2002)
    dref = T._updates(D2, list(D2), d0)
    f, c = T.frob(T._updates(None, list(D2), d0, res[0]["D2"]), dref)
    f32, _ = T.frob(T._updates(D232, list(D2), d0), dref)
    print(f"dp2 D2 update: rel-frob {f:.3e} (fp32 oracle {f32:.3e}) cos {c:.8f}")
    assert f <= 2 * f32 + 1e-3, (f, f32)
