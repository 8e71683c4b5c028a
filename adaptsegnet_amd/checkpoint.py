"""Checkpoint I/O.

* ``restore_from`` — the pretrained-weight remap of train_gta2cityscapes_multi.py:206-215:
  keys lose their first component (``Scale.layer5...`` -> ``layer5...``) and, for 19 classes,
  the 21-class ``layer5`` classifier is skipped; everything else is copied into a copy of the
  model's own state_dict, which is then loaded.
* ``save_snapshot`` / ``snapshot_step`` — the reference's snapshot files
  (:304-311 source-only, :482-493 single-level, :705-719 multi-level): plain
  ``torch.save(model.state_dict())`` with the reference's keys and NCHW shapes, named
  ``<snapshot_dir>/<level dir>/GTA5_<iter>.pth`` (+ ``_D1`` / ``_D2``), so snapshots are
  interchangeable with the reference's in both directions.
* ``save_resume`` / ``load_resume`` — what the reference lacks: one file with the three
  models, the SGD momentum buffers and Adam moments / step counts (keyed by parameter name, in
  the reference layout, like torch.optim state) and the iteration, so a run continues exactly.

Every load uses ``torch.load(..., weights_only=True)``.
"""
from __future__ import annotations

import os
import os.path as osp

import torch

LEVEL_DIRS = {"single-level": "single_level", "multi-level": "multi_level", "source-only": "source_only"}


def restore_from(model, saved_state_dict, num_classes: int = 19):
    """train_gta2cityscapes_multi.py:206-215 applied to an already-loaded state dict."""
    new_params = model.state_dict().copy()
    for i in saved_state_dict:
        i_parts = i.split(".")
        if not num_classes == 19 or not i_parts[1] == "layer5":
            new_params[".".join(i_parts[1:])] = saved_state_dict[i]
    model.load_state_dict(new_params)
    return model


def load_restore(model, path: str, num_classes: int = 19):
    """``torch.load(args.restore_from)`` (local file; the http model_zoo path needs network)."""
    return restore_from(model, torch.load(path, map_location="cpu", weights_only=True), num_classes)


def snapshot_paths(snapshot_dir: str, level: str, tag) -> dict:
    d = osp.join(snapshot_dir, LEVEL_DIRS[level])
    return {"G": osp.join(d, "GTA5_" + str(tag) + ".pth"),
            "D1": osp.join(d, "GTA5_" + str(tag) + "_D1.pth"),
            "D2": osp.join(d, "GTA5_" + str(tag) + "_D2.pth")}


def _cpu_state(m):
    return {k: v.detach().cpu() for k, v in m.state_dict().items()}


def save_snapshot(trainer, snapshot_dir: str, tag) -> dict:
    """Write the reference's snapshot files for ``trainer`` (D1 only in multi-level)."""
    paths = snapshot_paths(snapshot_dir, trainer.cfg.level, tag)
    os.makedirs(osp.dirname(paths["G"]), exist_ok=True)
    torch.save(_cpu_state(trainer.model), paths["G"])
    if trainer.cfg.level == "multi-level" and trainer.D1 is not None:
        torch.save(_cpu_state(trainer.D1), paths["D1"])
    if trainer.D2 is not None:
        torch.save(_cpu_state(trainer.D2), paths["D2"])
    return paths


def snapshot_step(trainer, snapshot_dir: str, i_iter: int, save_pred_every: int, num_steps_stop: int) -> bool:
    """The end-of-iteration snapshot logic (:482-493 / :705-719).  Returns True when training
    stops (the final ``GTA5_<num_steps_stop>`` snapshot was written)."""
    if i_iter >= num_steps_stop - 1:
        save_snapshot(trainer, snapshot_dir, num_steps_stop)
        return True
    if i_iter % save_pred_every == 0 and i_iter != 0:
        save_snapshot(trainer, snapshot_dir, i_iter)
    return False


def _arena_names(model):
    """Arena index -> the model's state_dict key of that parameter."""
    name_of = {id(p): n for n, p in model.named_parameters()}
    model._ensure_arena(next(model.parameters()).device)
    return [name_of[id(p)] for p in model.arena.params]


def save_resume(trainer, path: str, i_iter: int) -> None:
    out = {"i_iter": int(i_iter), "level": trainer.cfg.level}
    for key, m, opt in (("G", trainer.model, trainer.opt), ("D1", trainer.D1, trainer.opt_D1),
                        ("D2", trainer.D2, trainer.opt_D2)):
        if m is None:
            continue
        out[key] = _cpu_state(m)
        out["opt_" + key] = opt.state_dict(_arena_names(m))
    os.makedirs(osp.dirname(osp.abspath(path)), exist_ok=True)
    torch.save(out, path)


def load_resume(trainer, path: str) -> int:
    """Restore models and optimiser states; returns the iteration to continue from."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if ck["level"] != trainer.cfg.level:
        raise ValueError(f"checkpoint is {ck['level']}, trainer is {trainer.cfg.level}")
    for key, m, opt in (("G", trainer.model, trainer.opt), ("D1", trainer.D1, trainer.opt_D1),
                        ("D2", trainer.D2, trainer.opt_D2)):
        if m is None:
            continue
        names = _arena_names(m)
        m.load_state_dict(ck[key])
        opt.load_state_dict(ck["opt_" + key], names)
    return int(ck["i_iter"]) + 1
