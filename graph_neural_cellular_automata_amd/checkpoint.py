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


def pool_rng_states(pool) -> dict | None:
    """Every rank's private slot-index stream of a sharded ``SamplePool``, as
    ``{"world": W, "ranks": {rank: state}}``.  Collective when ``torch.distributed`` is initialised
    with the pool's world (every rank must call it; then every rank gets the whole map); otherwise
    only this process's rank is in the map.  None for an unsharded pool (it uses the global stream,
    which is the caller's to save)."""
    if pool is None or pool.rng_state() is None:
        return None
    import torch.distributed as dist
    mine = pool.rng_state()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() == pool.world > 1:
        got = [None] * pool.world
        dist.all_gather_object(got, (pool.rank, mine))
        return {"world": pool.world, "ranks": {int(r): st for r, st in got}}
    return {"world": pool.world, "ranks": {pool.rank: mine}}


def save_checkpoint(ckpt_dir, tag, model, optimizer, scheduler, epoch, global_step, config=None,
                    *, latest: bool = False, pool=None, pool_states: dict | None = None) -> str:
    """Write ``<ckpt_dir>/nca_<tag>.pt`` (and ``nca_latest.pt`` when ``latest``).  The private
    slot-index streams of a sharded ``SamplePool`` are saved too (``pool_rng_state``, an extra key
    the reference trainer ignores), per rank, so a resumed run continues EACH rank's sequence:
    pass ``pool_states`` from ``pool_rng_states(pool)`` (called on every rank; then only rank 0
    needs to save), or ``pool`` to store this process's rank only."""
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
    if pool_states is None and pool is not None:
        pool_states = pool_rng_states(pool) if pool.world == 1 else \
            {"world": pool.world, "ranks": {pool.rank: pool.rng_state()}}
    if pool_states is not None:
        payload["pool_rng_state"] = pool_states
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
    saved = payload.get("pool_rng_state")
    if pool is not None and saved is not None and pool.rng_state() is not None:
        if isinstance(saved, dict) and "ranks" in saved:
            ranks = {int(r): st for r, st in saved["ranks"].items()}
            if int(saved.get("world", -1)) != pool.world:
                print(f"[warn] pool streams were saved for world {saved.get('world')}, this run has "
                      f"world {pool.world}: the pool keeps its fresh stream", flush=True)
            elif pool.rank not in ranks:
                print(f"[warn] no saved pool stream for rank {pool.rank}: the pool keeps its fresh "
                      f"stream", flush=True)
            else:
                pool.set_rng_state(ranks[pool.rank])
        else:   # a single unlabelled stream (older checkpoints): its world size is not recorded, so
                # the sharding it was drawn for may differ (a one-rank pool has no private stream)
            print(f"[warn] checkpoint holds one unlabelled pool stream of an unknown world size: rank "
                  f"{pool.rank} of {pool.world} keeps its fresh stream", flush=True)
    return int(payload.get("epoch", 0)) + 1
