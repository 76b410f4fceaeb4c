"""Batch sharding of a rollout across ranks (one process per GPU).

Samples are independent (GroupNorm and the pooled logits are per sample), so a
rollout shards by contiguous sample ranges with no collective on the data path.  Everything the
ranks must agree on is derived from shared seeds:
  * per-step offsets: the same Python ``random.Random(seed)`` stream on every rank;
  * fire masks: the counter RNG keyed by GLOBAL sample index (``sample_base`` = first global
    index of the shard), so the union of the shards equals the unsharded rollout bit for bit.
"""
from __future__ import annotations

import random


def shard_range(global_batch: int, rank: int, world: int) -> tuple[int, int]:
    """[start, stop) of this rank's contiguous slice (sizes differ by at most one)."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def offsets_for_steps(seed: int, table, k: int, steps: int):
    """The per-step offset draws every rank makes identically (one random.sample per step, the
    reference's RNG call, graph_augmentation.py:120-121)."""
    rr = random.Random(seed)
    k = min(k, len(table))
    return [rr.sample(table, k) if k > 0 else [] for _ in range(steps)]
