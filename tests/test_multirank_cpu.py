"""world_size-2 gloo run of the sharded rollout logic on the CPU (no GPU): each rank rolls its
shard with the oracle (float64) using the shared offset draws and the global-index fire hash;
the all-gathered result must equal the single-process rollout bit for bit."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from graph_neural_cellular_automata_amd.modules.graph_augmentation import GraphAugmentation
from graph_neural_cellular_automata_amd.sharding import offsets_for_steps, shard_range
from oracle import nca_oracle as O
from tests.golden_io import Case

B, H, STEPS, SEED = 4, 16, 3, 42   # B even: gloo all_gather needs equal shards


def _rollout(x, base, p, cfg, offs):
    for t, chosen in enumerate(offs):
        fm = O.hash_fire_mask(SEED, t, base, x.shape[0], H, H, 0.5).astype(np.float64)
        x = O.nca_step(x, p, cfg, chosen=chosen, fire_mask=fm)
    return x


def _setup():
    c = Case("graph_torus_latest_grown_b1_72")
    p = {k: v.astype(np.float64) for k, v in c.weights.items()}
    rng = np.random.default_rng(0)
    x = rng.random((B, 16, H, H))
    offs = offsets_for_steps(SEED, GraphAugmentation._build_offsets(4), 8, STEPS)
    return x, p, c.cfg(), offs


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, p, cfg, offs = _setup()
    s, e = shard_range(B, rank, world)
    mine = torch.from_numpy(_rollout(x[s:e], s, p, cfg, offs))
    sizes = [shard_range(B, r, world) for r in range(world)]
    bufs = [torch.zeros(b - a, 16, H, H, dtype=torch.float64) for a, b in sizes]
    dist.all_gather(bufs, mine)
    if rank == 0:
        q.put(torch.cat(bufs).numpy())
    dist.destroy_process_group()


def test_shard_range_covers_batch():
    for world in (1, 2, 3, 8):
        for gb in (0, 1, 7, 1024):
            rs = [shard_range(gb, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == gb
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


def test_two_rank_gloo_rollout_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    x, p, cfg, offs = _setup()
    ref = _rollout(x, 0, p, cfg, offs)
    np.testing.assert_array_equal(got, ref)
