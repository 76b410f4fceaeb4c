"""Checkpoint round trip in the graph trainer's format.

Payload (``train_graph_augmented_nca.py:255-266``): ``{epoch, model_state, optimizer_state,
scheduler_state, config, param_count, global_step}``; file names ``nca_<tag>.pt`` plus the rolling
``nca_latest.pt``.  Resume (``:196-237``) scans the same candidates in the same order and keeps
the one with the largest (epoch, global_step).  The module's ``state_dict`` keys are the
reference's, so checkpoints move both ways between the reference trainer and this package.

Difference kept on purpose: files are read with ``torch.load(weights_only=True)`` (the payload
holds only tensors, numbers, strings, lists, dicts and None, so nothing is lost); a file that
only an unpickling loader could read is skipped like an unreadable one.
"""
from __future__ import annotations

import glob
import os
import re

import torch


def count_parameters(model) -> int:
    """Trainable parameter count (``utils/utility_functions.py:5-7``)."""
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def _epoch_num(name: str) -> int:
    m = re.search(r"epoch(\d+)", name)
    return int(m.group(1)) if m else -1


def save_checkpoint(ckpt_dir, tag, model, optimizer, scheduler, epoch, global_step, config=None,
                    *, latest: bool = False, pool=None) -> str:
    """Write ``<ckpt_dir>/nca_<tag>.pt`` (and ``nca_latest.pt`` when ``latest``).  ``pool``: a
    sharded ``SamplePool`` whose private slot-index stream is saved too (``pool_rng_state``), so a
    resumed run continues its sequence (an extra key; the reference trainer ignores it)."""
    os.makedirs(ckpt_dir, exist_ok=True)
    payload = {
        "epoch": int(epoch),
        "model_state": model.state_dict(),
        "optimizer_state": optimizer.state_dict(),
        "scheduler_state": scheduler.state_dict() if scheduler is not None else None,
        "config": config,
        "param_count": count_parameters(model),
        "global_step": int(global_step),
    }
    if pool is not None and pool.rng_state() is not None:
        payload["pool_rng_state"] = pool.rng_state()
    path = os.path.join(ckpt_dir, f"nca_{tag}.pt")
    torch.save(payload, path)
    if latest:
        torch.save(payload, os.path.join(ckpt_dir, "nca_latest.pt"))
    return path


def pick_resume(ckpt_dir):
    """(path, payload) of the newest readable checkpoint, or (None, None)."""
    cand = []
    latest = os.path.join(ckpt_dir, "nca_latest.pt")
    if os.path.exists(latest):
        cand.append(latest)
    cand += sorted(glob.glob(os.path.join(ckpt_dir, "nca_epoch*_final.pt")))
    cand += sorted(glob.glob(os.path.join(ckpt_dir, "nca_*_last.pt")))
    cand += sorted(glob.glob(os.path.join(ckpt_dir, "nca_crash_ep*.pt")))
    cand += sorted(glob.glob(os.path.join(ckpt_dir, "nca_epoch*.pt")), key=_epoch_num)
    best_path, best_payload, best = None, None, (-1, -1)
    for p in cand:
        try:
            payload = torch.load(p, map_location="cpu", weights_only=True)
            ep = int(payload.get("epoch", -1))
            gs = int(payload.get("global_step", ep))
        except Exception:
            continue
        if ep > best[0] or (ep == best[0] and gs > best[1]):
            best, best_path, best_payload = (ep, gs), p, payload
    return best_path, best_payload


def load_checkpoint(payload, model, optimizer=None, scheduler=None, pool=None) -> int:
    """Restore model (``strict=False``), optimizer and scheduler state as the trainer's resume
    does (an incompatible optimizer/scheduler state is reported and skipped), and a sharded pool's
    slot-index stream when the payload has one.  Returns the epoch to start from."""
    missing, unexpected = model.load_state_dict(payload["model_state"], strict=False)
    if missing:
        print(f"[resume] missing model keys: {missing}", flush=True)
    if unexpected:
        print(f"[resume] unexpected model keys: {unexpected}", flush=True)
    if optimizer is not None and payload.get("optimizer_state") is not None:
        try:
            optimizer.load_state_dict(payload["optimizer_state"])
        except Exception as e:
            print(f"[warn] optimizer state not compatible, reinitializing: {e}", flush=True)
    if scheduler is not None and payload.get("scheduler_state") is not None:
        try:
            scheduler.load_state_dict(payload["scheduler_state"])
        except Exception as e:
            print(f"[warn] scheduler state not compatible, reinit: {e}", flush=True)
    if pool is not None and payload.get("pool_rng_state") is not None:
        pool.set_rng_state(payload["pool_rng_state"])
    return int(payload.get("epoch", 0)) + 1
