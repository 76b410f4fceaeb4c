"""The device-resident SamplePool against the reference's list-of-tensors semantics
(src/training/pool.py:5-42, restated here as a 10-line list implementation): same slot contents,
same random.sample draws, same replace behaviour; the sharded pool holds the right slice and
keeps the seed RNG stream in step with the unsharded one."""
import random

import torch

from graph_neural_cellular_automata_amd.pool import SamplePool


def _seed_fn(batch_size=1):
    """The graph trainer's seed (train_graph_augmented_nca.py:108-114) on a 12x12 canvas."""
    g = torch.zeros(batch_size, 8, 12, 12)
    g[:, 3:4, 6, 6] = 1.0
    g[:, 4:, 6, 6] = 0.01 * torch.randn_like(g[:, 4:, 6, 6])
    return g


class _ListPool:
    def __init__(self, n, seed_fn):
        self.pool = [seed_fn(batch_size=1).squeeze(0) for _ in range(n)]

    def sample(self, b):
        idx = random.sample(range(len(self.pool)), b)
        return idx, torch.stack([self.pool[i].clone() for i in idx])

    def replace(self, idx, new):
        for i, s in zip(idx, new):
            self.pool[i] = s.detach().clone()


def test_pool_matches_list_semantics():
    torch.manual_seed(0)
    ref = _ListPool(20, _seed_fn)
    torch.manual_seed(0)
    pool = SamplePool(20, _seed_fn, device="cpu")
    assert torch.equal(torch.stack(ref.pool), pool.states)
    for it in range(5):
        random.seed(it)
        i1, b1 = ref.sample(6)
        random.seed(it)
        i2, b2 = pool.sample(6)
        assert i1 == i2 and torch.equal(b1, b2)
        new = b1 + it + 1.0
        ref.replace(i1, new)
        pool.replace(i2, new)
        b2.add_(100.0)   # the sampled batch is a copy
        assert torch.equal(torch.stack(ref.pool), pool.states)


def test_sharded_pool_slices_and_rng_stream():
    torch.manual_seed(1)
    full = SamplePool(10, _seed_fn)
    after_full = torch.randn(3)
    parts = []
    for r in range(3):
        torch.manual_seed(1)
        p = SamplePool(10, _seed_fn, shard=(r, 3))
        assert torch.equal(torch.randn(3), after_full)   # every rank consumed the same seeds
        parts.append(p)
    assert [len(p) for p in parts] == [4, 3, 3]
    assert torch.equal(torch.cat([p.states for p in parts]), full.states)


def test_sharded_pool_sampling_keeps_global_stream():
    """Ranks whose slices differ in length must not desynchronise the global random stream (the
    per-step offset draws are shared by every rank)."""
    parts = [SamplePool(10, _seed_fn, shard=(r, 3)) for r in range(3)]
    after = []
    for p in parts:
        random.seed(5)
        idx, batch = p.sample(3)
        assert len(set(idx)) == 3 and all(0 <= i < len(p) for i in idx)
        assert batch.shape[0] == 3
        after.append(random.random())
    assert after[0] == after[1] == after[2]
