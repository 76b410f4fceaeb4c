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


def test_sharded_pool_stream_follows_user_seed_and_checkpoints(tmp_path):
    """The private slot-index stream of a sharded pool depends on the user's random.seed (read from
    the global state, not consumed), differs per rank, and survives a checkpoint round trip."""
    import torch.nn as nn

    from graph_neural_cellular_automata_amd.checkpoint import load_checkpoint, save_checkpoint

    def draws(seed, rank):
        random.seed(seed)
        p = SamplePool(12, _seed_fn, shard=(rank, 2))
        after = random.random()
        return [p.sample(3)[0] for _ in range(4)], after, p

    a, after_a, _ = draws(1, 0)
    b, after_b, _ = draws(2, 0)
    c, _, _ = draws(1, 1)
    random.seed(1)
    assert after_a == random.random()   # building the sharded pool consumed nothing
    assert a != b and a != c
    # checkpoint: resume continues the sequence
    _, _, p = draws(7, 1)
    p.sample(3)
    model = nn.Linear(2, 2)
    opt = torch.optim.Adam(model.parameters())
    save_checkpoint(str(tmp_path), "epoch1", model, opt, None, 1, 10, pool=p)
    expect = [p.sample(3)[0] for _ in range(3)]
    _, _, q = draws(99, 1)
    payload = torch.load(str(tmp_path / "nca_epoch1.pt"), weights_only=True)
    load_checkpoint(payload, model, opt, None, pool=q)
    assert [q.sample(3)[0] for _ in range(3)] == expect
