"""Parity at BASELINE's full geometries (batch 1, and each config's own bench batch): the
large-grid kernel paths end to end.

Every other model-level test runs at 41x57-class sizes, where most convs split K and go
through the slab reduce; at 1024x512 / 1280x720 the layer3/4 convs run unsplit with the
in-kernel epilogue.  Two checks:

1. test_fullres_step_vs_oracle — ONE iteration of the adversarial step on the HIP engine vs
   the fp32 oracle (oracle/reference_torch.py: stock PyTorch CPU ops, the reference's own
   arithmetic and dtype) from identical deterministic weights and inputs:
     c2 geometry: single-level Vanilla, source and target 1024x512 (train:385-461);
     c3 geometry: multi-level Vanilla, source 1280x720, target 1024x512 (train:578-679).
   Losses within 1e-3 relative (train- and eval-mode BN); per-group parameter-update cosine
   >= 0.99 in eval-mode BN (well conditioned) and >= 0.97 in train-mode BN (the
   reference's own fp32 weight gradients scatter by 4-5 % at random init).

2. test_fullres_trajectory — five iterations on one fixed batch vs the committed loss
   trajectories of the REFERENCE modules themselves (tests/golden/trajectory_goldens.npz,
   gen_trajectory.py, fp32 CPU).  This pins the bench's double-digit loss_seg2 as the
   reference's own random-init behaviour (the duplicated-parameter SGD of
   get_1x_lr_params_NOscale applies each trunk update 3-4x, deeplab_multi.py:216-222).
   Iteration 0 within 1e-3; later iterations within max(4x the reference's own 8-vs-3-thread
   spread, the stated floor) — the train-BN trajectory is chaotic at random init.  The CPU
   thread spread understates that chaos (both runs share MKL's algorithms), so train-BN runs
   also measure the HIP path's own sensitivity: the same five steps under a second fp32-accurate
   summation order (engine.X3_FWD_TERMS 1: layers 3-4 conv2 on the term-image kernels, whose
   weight gradient splits K differently), and allow 2x that divergence.  Round 6 evidence
   (profiles/r6/trajectory_sensitivity.txt): c3_train's two orders agree within 0.2 % up to
   iteration 3 and end 16 % apart at iteration 4 (loss_seg2 23.57 vs 28.18; reference 27.78).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import reference_torch as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
HERE = os.path.dirname(os.path.abspath(__file__))

GEOMS = {
    "c2": ("single-level", (1024, 512), (1024, 512)),
    "c3": ("multi-level", (1280, 720), (1024, 512)),
}


def _batch(src, tgt, batch=1):
    xs = torch.from_numpy(R.det_images((batch, 3, src[1], src[0]), 11)).float()
    lab = torch.from_numpy(R.det_labels((batch, src[1], src[0]), 12))
    xt = torch.from_numpy(R.det_images((batch, 3, tgt[1], tgt[0]), 13)).float()
    return xs, lab, xt


def _sd(specs, seed):
    return {k: torch.from_numpy(v.copy()) if v.dtype == np.int64 else torch.from_numpy(v.copy()).float()
            for k, v in R.det_state(specs, seed).items()}


def _hip_trainer(level, src, tgt, bn_train, gan="Vanilla"):
    from adaptsegnet_amd.model import DeeplabMulti, FCDiscriminator
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    m = DeeplabMulti(num_classes=19)
    m.load_state_dict(_sd(R.g_specs(), 1338))
    m = m.to(DEV).train(bn_train)
    d1 = FCDiscriminator(num_classes=19)
    d1.load_state_dict(_sd(R.d_specs(), 2001))
    d2 = FCDiscriminator(num_classes=19)
    d2.load_state_dict(_sd(R.d_specs(), 2002))
    d1, d2 = d1.to(DEV), d2.to(DEV)
    tr = AdaptSegTrainer(m, d1 if level == "multi-level" else None, d2,
                         StepConfig(level=level, gan=gan, input_size=src, input_size_target=tgt))
    return tr, m, d1, d2


def _cos(a, b):
    return float(F.cosine_similarity(a.flatten(), b.flatten(), dim=0))


# (batch 1: train-mode BN; the eval-BN batch-1 runs were subsumed by the bench-batch ones below,
# which check the same kernels on larger grids with the well-conditioned eval-BN bounds, and so
# was c2's train-BN batch-1 run by its B=4 one — dropped in round 6 to keep the GPU suite inside
# its time limit)
@pytest.mark.parametrize("bn_train", [True], ids=["trainBN"])
@pytest.mark.parametrize("geom", ["c3"])
def test_fullres_step_vs_oracle(geom, bn_train):
    _step_vs_oracle(geom, bn_train, "Vanilla", 1e-3)


# BASELINE's own per-GPU batch of each config (bench.py CONFIGS): the engine's batch-dependent
# planning (row-tile statistics, split-K counts, bf16_only copy skipping, kernel selection by
# grid size) runs end to end at exactly the shapes the bench lines are measured on
BENCH_BATCH = {"c2": 4, "c3": 2}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("geom,bn_train", [("c2", True), ("c3", False)], ids=["c2-trainBN", "c3-evalBN"])
def test_fullres_bench_batch_step_vs_oracle(geom, bn_train):
    """test_fullres_step_vs_oracle at the bench's batch: c2 single-level Vanilla at B=4
    (train:385-461), c3 multi-level Vanilla at B=2 (train:578-679); the same bounds as batch 1
    (losses within 1e-3, update cosine >= 0.97 train BN / 0.99 eval BN).  Dropped in round 6 for
    the suite's time limit: c3's train-BN run at B=2 (its batch-1 run stays) and c2's eval-BN run
    at B=4 (the bench runs train-mode BN, checked at B=4 here; eval-mode BN is checked at c3's
    bench batch and by test_model_gpu.py's eval-BN steps)."""
    _step_vs_oracle(geom, bn_train, "Vanilla", 1e-3, batch=BENCH_BATCH[geom])


def test_fullres_fused_bn_sums_match_unfused(monkeypatch):
    """engine.BN_SUMS (the BN1 / BN2 backward reductions fused into the producing data
    gradients' epilogues) at the c2 geometry, train-mode BN, batch 1: the losses are the
    forward's and stay bit-identical; the parameter updates differ only by the reductions'
    summation order (every group's update cosine >= 0.9999 against the unfused step); and with
    the switch on, the step against the fp32 oracle holds test_fullres_step_vs_oracle's bounds."""
    from adaptsegnet_amd import engine
    level, src, tgt = GEOMS["c2"]
    xs, lab, xt = _batch(src, tgt)
    runs = []
    for mode in (0, 3):
        monkeypatch.setattr(engine, "BN_SUMS", mode)
        tr, m, d1, d2 = _hip_trainer(level, src, tgt, True)
        got = tr.step(0, [(xs.to(DEV), lab.to(DEV), xt.to(DEV))]).values()
        runs.append((got, {k: v.detach().cpu().double() for k, v in m.state_dict().items()},
                     {k: v.detach().cpu().double() for k, v in d2.state_dict().items()}))
    (l0, g0, dd0), (l1, g1, dd1) = runs
    assert l0 == l1, (l0, l1)
    init = _sd(R.g_specs(), 1338)
    keys = [k for k in g0 if g0[k].is_floating_point() and not k.startswith("layer5") and "running" not in k]
    u0 = torch.cat([(g0[k] - init[k].double()).flatten() for k in keys])
    u1 = torch.cat([(g1[k] - init[k].double()).flatten() for k in keys])
    c = _cos(u1, u0)
    print(f"fused BN sums: G update cosine vs unfused {c:.8f}")
    assert c >= 0.9999, c
    dinit = _sd(R.d_specs(), 2002)
    cd = _cos(torch.cat([(dd1[k] - dinit[k].double()).flatten() for k in dd1]),
              torch.cat([(dd0[k] - dinit[k].double()).flatten() for k in dd0]))
    assert cd >= 0.9999, cd
    _step_vs_oracle("c2", True, "Vanilla", 1e-3)


@pytest.fixture
def bf16_math():
    from adaptsegnet_amd import kernels as K
    K.set_conv_math(K.MATH_BF16)
    yield K
    K.set_conv_math(K.MATH_F32X3)   # the library default


@pytest.mark.parametrize("bn_train", [True, False], ids=["trainBN", "evalBN"])
def test_fullres_c5_bf16_step_vs_oracle(bf16_math, bn_train):
    """BASELINE config c5's program (multi-level LS-GAN, bf16 conv math, train:578-679) at its own
    geometry — source 1280x720, target 1024x512, batch 1 — against the fp32 oracle with bf16
    activation storage (every Bottleneck conv / BN / block output rounded to bf16 as stored,
    R.bf16_activation_storage; the engine's torch.autocast-style storage): the bf16 LDS-DMA
    kernels on bf16 activations, with the fp32 tensors that only those kernels read never
    written (engine.bf16_only), run unsplit at this size.  Losses within
    2e-2 relative (bf16 operand rounding, ~2^-9 per operand through ~100 layers); eval BN: every
    update cosine >= 0.99.  Train BN: the trunk update is not comparable with the fp32 oracle's
    at all — the reference's OWN arithmetic with bf16 conv operands moves it to cosine -0.002
    (experiments/bf16_trainbn_sensitivity.py, profiles/r3/bf16_trainbn_sensitivity.txt: the
    random-init train-BN trunk gradient is chaotic under bf16 rounding, the losses and heads are
    not), so the train-BN check is the losses, the heads' update (>= 0.97; the emulation: 0.9998)
    and the discriminators' (>= 0.85: Adam's first step is nearly sign(g); the emulation 0.92)."""
    _step_vs_oracle("c3", bn_train, "LS", 2e-2, trunk=not bn_train, d_bound=0.85 if bn_train else None,
                    act_bf16=True)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("bn_train", [False], ids=["evalBN"])
def test_fullres_c5_bench_batch_step_vs_oracle(bf16_math, bn_train):
    """test_fullres_c5_bf16_step_vs_oracle at BASELINE c5's batch/GPU 4 (the bench line's shape):
    the same bounds (losses within 2e-2; eval BN every update cosine >= 0.99).  Eval BN only: its
    train-BN twin pinned only the losses, heads and discriminators (the trunk is chaotic under
    bf16 rounding at random init) and cost 54 s of the suite; the train-BN c5 program stays
    checked at batch 1 (test_fullres_c5_bf16_step_vs_oracle[trainBN])."""
    _step_vs_oracle("c3", bn_train, "LS", 2e-2, trunk=not bn_train, d_bound=0.85 if bn_train else None,
                    act_bf16=True, batch=4)


def test_fullres_c5_bf16_skipping_fp32_copies_is_bitwise_neutral(bf16_math, monkeypatch):
    """engine.bf16_only at the c5 geometry: one train-BN multi-level LS step with and without the
    skipping of fp32 activations gives bitwise the same losses and parameters (a skipped tensor is
    never read by the full-size kernel variants: tests/test_copy_plan_cpu.py lists those)."""
    from adaptsegnet_amd import engine
    level, src, tgt = GEOMS["c3"]
    xs, lab, xt = _batch(src, tgt)
    b = [(xs.to(DEV), lab.to(DEV), xt.to(DEV))]
    g = bf16_math.ConvGeom(256, 256, 3, 3, 1, (2,), (2,))
    assert engine.bf16_only(g, 1, 90, 160, (0, 1, 2))   # layer3.conv2 at 1280x720 reads only copies
    runs = []
    for skip in (True, False):
        if not skip:
            monkeypatch.setattr(engine, "bf16_only", lambda *a, **kw: False)
        tr, m, d1, d2 = _hip_trainer(level, src, tgt, True, gan="LS")
        vals = tr.step(0, b).values()
        torch.cuda.synchronize()
        runs.append((vals, [{k: v.detach().cpu().clone() for k, v in mm.state_dict().items()} for mm in (m, d1, d2)]))
    (va, sa), (vb, sb) = runs
    assert va == vb, (va, vb)
    for da, db in zip(sa, sb):
        for k in da:
            assert torch.equal(da[k], db[k]), k


@pytest.mark.timeout(600)
@pytest.mark.parametrize("batch", [1, 8], ids=["B1", "B8"])
def test_fullres_c4_vgg_step_vs_oracle(batch):
    """BASELINE config c4's program at its own geometry: DeeplabVGG (model/deeplab_vgg.py:24-54)
    single-level Vanilla step (train:385-461, the map upsampled by the caller's interp), source and
    target 1024x512, batch 1 and BASELINE's batch 8, against the fp32 oracle (R.vgg_forward, the restatement: DeeplabVGG
    is unimportable here, so the composition is pinned by the restatement and the per-op goldens,
    SURVEY.md §8c) from identical weights and inputs.  At this size the conv5 / fc6 / fc7 products
    run unsplit with the in-kernel epilogue.  Losses within 1e-3 relative; the generator's update
    (one SGD group, optim_parameters = parameters()) and D2's at cosine >= 0.99 (VGG has no BN:
    the update is well conditioned); the classifier branches the forward never reaches keep no
    gradient and no update in both."""
    from adaptsegnet_amd.model import DeeplabVGG, FCDiscriminator
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    src = tgt = (1024, 512)
    xs, lab, xt = _batch(src, tgt, batch)
    cfg = dict(level="single-level", gan="Vanilla", input_size=src, input_size_target=tgt, gen="vgg")
    st = R.det_state(R.vgg_specs(), 4244)
    P = R.to_torch(st, dtype=torch.float32, trainable=lambda k: True)
    D2 = R.to_torch(R.det_state(R.d_specs(), 2002), dtype=torch.float32, trainable=lambda k: True)
    opts = R.make_optimizers(P, None, D2, R.DEFAULT_CFG | cfg)
    ref = R.oracle_step(P, None, D2, opts, cfg, 0, [(xs, lab, xt)])
    m = DeeplabVGG(19)
    m.load_state_dict({k: torch.from_numpy(v.copy()).float() for k, v in st.items()})
    m = m.to(DEV)
    d2 = FCDiscriminator(num_classes=19)
    d2.load_state_dict(_sd(R.d_specs(), 2002))
    d2 = d2.to(DEV)
    tr = AdaptSegTrainer(m, None, d2, StepConfig(level="single-level", input_size=src, input_size_target=tgt))
    got = tr.step(0, [(xs.to(DEV), lab.to(DEV), xt.to(DEV))]).values()
    for k, v in ref.items():
        print(f"c4 B={batch} {k}: hip={got[k]:.6f} oracle={v:.6f}")
        assert abs(got[k] - v) <= 1e-3 * abs(v) + 1e-6, (k, got[k], v)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    used = [k for k in P if not k.startswith(("classifier.conv2d_list.2", "classifier.conv2d_list.3"))]
    for k in P:
        if k not in used:
            assert torch.equal(sd[k].double(), torch.from_numpy(st[k]).float().double()), k
            assert torch.equal(P[k].detach().double(), torch.from_numpy(st[k]).float().double()), k
    u_ref = torch.cat([(P[k].detach().double() - torch.from_numpy(st[k])).flatten() for k in used])
    u_hip = torch.cat([(sd[k].double() - torch.from_numpy(st[k])).flatten() for k in used])
    c = _cos(u_hip, u_ref)
    print(f"c4 G update cosine {c:.6f}")
    assert c >= 0.99, c
    d0 = R.det_state(R.d_specs(), 2002)
    dsd = d2.state_dict()
    u_ref = torch.cat([(D2[k].detach().double() - torch.from_numpy(d0[k])).flatten() for k in D2])
    u_hip = torch.cat([(dsd[k].double().cpu() - torch.from_numpy(d0[k])).flatten() for k in D2])
    c = _cos(u_hip, u_ref)
    print(f"c4 D2 update cosine {c:.6f}")
    assert c >= 0.99, c


def test_c1_forward_crossentropy2d_vs_oracle():
    """BASELINE config c1 at its own shape: DeeplabMulti forward (train-mode BN, single head)
    + utils/loss.py CrossEntropy2d on one 1x3x321x321 tensor (model/deeplab_multi.py:174-194,
    utils/loss.py:14-36) against the fp64 oracle: outputs within 1e-3 of max|ref|, loss within
    1e-3 relative; the same with eval-mode BN."""
    from adaptsegnet_amd.model import DeeplabMulti
    from adaptsegnet_amd.utils.loss import CrossEntropy2d
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    x = torch.from_numpy(R.det_images((1, 3, 321, 321), 5))
    lab = torch.from_numpy(R.det_labels((1, 321, 321), 6))
    G = R.to_torch(R.det_state(R.g_specs(), 1338), trainable=R.g_trainable)
    m = DeeplabMulti(num_classes=19)
    m.load_state_dict(_sd(R.g_specs(), 1338))
    m = m.to(DEV)
    for train in (True, False):
        with torch.no_grad():
            _, p2 = R.g_forward(G, x, (321, 321), train=train)
            l_ref = float(R.cross_entropy2d(p2, lab))
            m.train(train)
            _, q2 = m(x.float().to(DEV), (321, 321))
            loss = float(CrossEntropy2d()(q2, lab.to(DEV)))
        err = float((q2.double().cpu() - p2).abs().max() / p2.abs().max())
        print(f"c1 train={train}: forward rel err {err:.2e}, loss hip={loss:.6f} oracle={l_ref:.6f}")
        assert q2.shape == p2.shape == (1, 19, 321, 321)
        assert err < 1e-3
        assert abs(loss - l_ref) <= 1e-3 * abs(l_ref)


# one oracle step per (geometry, BN mode, GAN, storage, batch) per session: the full-size CPU
# steps dominate this module's time, and test_fullres_fused_bn_sums_match_unfused repeats
# test_fullres_step_vs_oracle[trainBN-c2]'s
_ORACLE_CACHE: dict = {}


def _oracle_step(geom, bn_train, gan, act_bf16, batch):
    key = (geom, bn_train, gan, act_bf16, batch)
    if key not in _ORACLE_CACHE:
        level, src, tgt = GEOMS[geom]
        xs, lab, xt = _batch(src, tgt, batch)
        cfg = dict(level=level, gan=gan, input_size=src, input_size_target=tgt)
        # oracle, fp32 on the host cores
        G = R.to_torch(R.det_state(R.g_specs(), 1338), dtype=torch.float32, trainable=R.g_trainable)
        D1 = R.to_torch(R.det_state(R.d_specs(), 2001), dtype=torch.float32, trainable=lambda k: True)
        D2 = R.to_torch(R.det_state(R.d_specs(), 2002), dtype=torch.float32, trainable=lambda k: True)
        opts = R.make_optimizers(G, D1 if level == "multi-level" else None, D2, R.DEFAULT_CFG | cfg)
        if act_bf16:
            with R.bf16_activation_storage():
                ref = R.oracle_step(G, D1, D2, opts, cfg, 0, [(xs, lab, xt)], bn_train=bn_train)
        else:
            ref = R.oracle_step(G, D1, D2, opts, cfg, 0, [(xs, lab, xt)], bn_train=bn_train)
        _ORACLE_CACHE[key] = (ref, G, D1, D2)
    return _ORACLE_CACHE[key]


def _step_vs_oracle(geom, bn_train, gan, tol, trunk=True, d_bound=None, act_bf16=False, batch=1):
    """act_bf16: the oracle stores the Bottleneck activations in bf16 as the engine's bf16
    program does (R.bf16_activation_storage).  batch: images per domain (the bench's own batch
    sizes: test_fullres_bench_batch_step_vs_oracle)."""
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    level, src, tgt = GEOMS[geom]
    xs, lab, xt = _batch(src, tgt, batch)
    ref, G, D1, D2 = _oracle_step(geom, bn_train, gan, act_bf16, batch)
    # HIP engine
    tr, m, d1, d2 = _hip_trainer(level, src, tgt, bn_train, gan=gan)
    got = tr.step(0, [(xs.to(DEV), lab.to(DEV), xt.to(DEV))]).values()
    for k, v in ref.items():
        print(f"{geom} B={batch} {gan} bn_train={bn_train} {k}: hip={got[k]:.6f} oracle={v:.6f}")
        assert abs(got[k] - v) <= tol * abs(v) + 1e-6, (k, got[k], v)
    # parameter updates (new - initial), per group
    g0 = R.det_state(R.g_specs(), 1338)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    groups = {"trunk": [], "heads": []}
    for k, t in G.items():
        if t.dtype.is_floating_point and t.requires_grad:
            if k.startswith("layer5") and level == "single-level":
                continue
            groups["heads" if k.startswith(("layer5", "layer6")) else "trunk"].append(k)
    bound = 0.97 if bn_train else 0.99
    for gname, keys in groups.items():
        if gname == "trunk" and not trunk:
            continue
        u_ref = torch.cat([(G[k].detach().double() - torch.from_numpy(g0[k])).flatten() for k in keys])
        u_hip = torch.cat([(sd[k].double() - torch.from_numpy(g0[k])).flatten() for k in keys])
        c = _cos(u_hip, u_ref)
        print(f"{geom} B={batch} bn_train={bn_train} G/{gname} update cosine {c:.6f}")
        assert c >= bound, (gname, c)
    for dname, dm, DD, seed in (("D1", d1, D1, 2001), ("D2", d2, D2, 2002)):
        if dname == "D1" and level == "single-level":
            continue
        d0 = R.det_state(R.d_specs(), seed)
        dsd = dm.state_dict()
        u_ref = torch.cat([(DD[k].detach().double() - torch.from_numpy(d0[k])).flatten() for k in DD])
        u_hip = torch.cat([(dsd[k].double().cpu() - torch.from_numpy(d0[k])).flatten() for k in DD])
        c = _cos(u_hip, u_ref)
        print(f"{geom} B={batch} bn_train={bn_train} {dname} update cosine {c:.6f}")
        assert c >= (d_bound or bound), (dname, c)


TRAJ_RUNS = {"c2_train": ("c2", True), "c2_eval": ("c2", False), "c3_train": ("c3", True)}
# floor of the later-iteration bound, relative to the loss: the eval-BN trajectory is smooth,
# the train-BN one chaotic at random init (see module docstring)
TRAJ_FLOOR = {"c2_train": 0.05, "c2_eval": 2e-3, "c3_train": 0.05}


@pytest.mark.parametrize("run", list(TRAJ_RUNS))
def test_fullres_trajectory(run):
    gold = np.load(os.path.join(HERE, "golden", "trajectory_goldens.npz"))
    ref8, ref3 = gold[f"{run}/threads8"], gold[f"{run}/threads3"]
    names = [str(s) for s in gold[f"{run}/names"]]
    geom, bn_train = TRAJ_RUNS[run]
    level, src, tgt = GEOMS[geom]
    xs, lab, xt = _batch(src, tgt)
    b = [(xs.to(DEV), lab.to(DEV), xt.to(DEV))]

    def trajectory():
        tr, *_ = _hip_trainer(level, src, tgt, bn_train)
        return [tr.step(it, b).values() for it in range(ref8.shape[0])]
    got_all = trajectory()
    alt_all = None
    if bn_train:   # the HIP path's own summation-order sensitivity (module docstring)
        from adaptsegnet_amd import engine
        prev = engine.X3_FWD_TERMS
        engine.X3_FWD_TERMS = 1 - prev
        try:
            alt_all = trajectory()
        finally:
            engine.X3_FWD_TERMS = prev
    for it in range(ref8.shape[0]):
        got = got_all[it]
        for j, k in enumerate(names):
            v, spread = float(ref8[it, j]), abs(float(ref8[it, j] - ref3[it, j]))
            own = abs(got[k] - alt_all[it][k]) if alt_all is not None else 0.0
            bound = 1e-3 * abs(v) if it == 0 else max(4 * spread, TRAJ_FLOOR[run] * abs(v), 2 * own)
            print(f"{run} iter{it} {k}: hip={got[k]:.5f} reference={v:.5f} (8 vs 3 threads {spread:.2e}, "
                  f"HIP summation orders {own:.2e})")
            assert abs(got[k] - v) <= bound + 1e-6, (run, it, k, got[k], v, bound)
