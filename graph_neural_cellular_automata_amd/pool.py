"""Device-resident sample pool, the caller-side data format of the path.

Mirror of the reference's ``SamplePool`` (``src/training/pool.py:5-42``) with the same
constructor, ``sample`` and ``replace`` (same argument meaning and the same Python ``random``
consumption), but the pool is ONE contiguous ``[P, C, H, W]`` device tensor instead of a list of
P separate tensors: ``sample`` is one ``index_select`` (the reference stacks B clones) and
``replace`` one ``index_copy_`` (the reference assigns B clones one by one).  On a 288 GB MI355X the
whole C4 pool (1024 x 16 x 72 x 72 fp32 = 340 MB) stays resident.

Multi-GPU (``shard=(rank, world)``): each rank keeps only its contiguous slice of the pool
(``sharding.shard_range``) and samples its share of the batch from it.  Every rank still calls
``seed_fn`` for all P samples, so the global RNG streams stay identical across ranks.  A sharded
pool draws its slot indices from its own ``random.Random``, not from the global stream: slices may
differ in length by one, and ``random.sample`` over different lengths consumes the stream
differently, which would desynchronise the per-step offset draws that every rank must share
(``sharding.py``).  That private stream is seeded from the global stream's STATE at construction
(read, not consumed: identical on every rank, and it follows the user's ``random.seed``) mixed
with the rank; ``rng_state()`` / ``set_rng_state()`` carry it through a checkpoint: every rank
calls ``checkpoint.pool_rng_states(pool)`` (collective over the pool's world), rank 0 saves the
result with ``save_checkpoint(..., pool_states=)``, and ``load_checkpoint(..., pool=)`` on each rank
restores that rank's own stream (``save_checkpoint(..., pool=)`` stores only the calling rank's).
"""
from __future__ import annotations

import hashlib
import random

import torch

from .sharding import shard_range


class SamplePool:
    def __init__(self, pool_size, seed_fn, device="cpu", *, shard: tuple[int, int] | None = None):
        """``seed_fn(batch_size=1)`` returns one seed state ([1,C,H,W] or [C,H,W]), called once per
        pool slot exactly as the reference does (pool.py:18)."""
        self.pool_size = int(pool_size)
        rank, world = shard if shard is not None else (0, 1)
        self.rank, self.world = int(rank), int(world)
        self.lo, self.hi = shard_range(self.pool_size, rank, world)
        seeds = []
        for i in range(self.pool_size):
            s = seed_fn(batch_size=1)
            if i >= self.lo and i < self.hi:
                seeds.append(s.reshape(s.shape[-3:]).to(device))
        self.states = torch.stack(seeds).contiguous() if seeds else torch.empty(0, device=device)
        # unsharded: the global stream, exactly as the reference; sharded: a private stream
        if world == 1:
            self._rng = random
        else:
            digest = hashlib.sha256(repr(random.getstate()).encode()).digest()
            self._rng = random.Random(int.from_bytes(digest[:8], "little") * 1_000_003 + rank * 1009 + world)

    def __len__(self):
        return self.states.shape[0]

    @property
    def pool(self):
        """The slots as a list of [C,H,W] views (the reference's attribute, for reading)."""
        return list(self.states.unbind(0))

    def sample(self, batch_size):
        """(idx, batch): ``random.sample`` over this pool's slots (pool.py:23-32) and a fresh
        [B,C,H,W] tensor (a copy: the pool is not modified through it)."""
        idx = self._rng.sample(range(len(self)), batch_size)
        sel = torch.as_tensor(idx, dtype=torch.long, device=self.states.device)
        return idx, self.states.index_select(0, sel)

    def rng_state(self):
        """The private slot-index stream's state (a sharded pool), else None (the global stream is
        the caller's to save).  JSON/torch.save-friendly (nested lists)."""
        if self._rng is random:
            return None
        v, st, g = self._rng.getstate()
        return [v, list(st), g]

    def set_rng_state(self, state):
        if state is not None and self._rng is not random:
            v, st, g = state
            self._rng.setstate((int(v), tuple(int(t) for t in st), g))

    def replace(self, idx, new_samples):
        """Write ``new_samples`` (detached) into slots ``idx`` (pool.py:34-42)."""
        sel = torch.as_tensor(list(idx), dtype=torch.long, device=self.states.device)
        self.states.index_copy_(0, sel, new_samples.detach().to(self.states.dtype))
