"""Rank bodies of the multi-rank GPU tests (tests/test_gpu_multirank.py).

Each function runs in a fresh process forked from the test session's forkserver (started in
tests/conftest.py before any GPU call, so no process that has initialised the GPU ever execs),
joins a world_size-2 gloo process group on 127.0.0.1, and drives the HIP path on cuda:0 (both
ranks share the one GPU of the test box; RCCL would refuse two ranks on one device, gloo carries
the host-side collectives).  Results go back through files / a queue to the parent, which holds
the single-process reference.
"""
from __future__ import annotations

import os
import random


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    return dev


# ---- the sharded rollout (BASELINE config 4's data path: 128 samples per GPU) -------------------
ROLL = dict(B=256, C=16, H=72, steps=12, seed=42, state_seed=1234, offset_seed=77,
            fixture="graph_torus_latest_grown_b1_72")


def roll_state(spec):
    """The global start state (CPU generator: the same bits in every process)."""
    import torch
    g = torch.Generator().manual_seed(spec["state_seed"])
    x = torch.rand(spec["B"], spec["C"], spec["H"], spec["H"], generator=g)
    x[:, 4:] = torch.randn(spec["B"], spec["C"] - 4, spec["H"], spec["H"], generator=g)
    return x


def roll_offsets(spec):
    from graph_neural_cellular_automata_amd.sharding import offsets_for_steps
    from oracle import nca_oracle as O   # only the row-major offset table (graph_augmentation.py:73-83)
    return offsets_for_steps(spec["offset_seed"], O.build_offsets(4), 8, spec["steps"])


def hip_rollout(spec, x, base, dev):
    """gnca_rollout_f32 of samples [base, base + len(x)) with the bench's knobs."""
    import numpy as np
    import torch

    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    from tests.golden_io import Case
    c = Case(spec["fixture"])
    wt = {k: torch.from_numpy(np.ascontiguousarray(v.astype(np.float32))).to(dev) for k, v in c.weights.items()}
    w, keep = S.make_weights(dict(
        perception=wt["perception.conv.weight"], w1=wt["update_net.0.weight"], b1=wt["update_net.0.bias"],
        w2=wt["update_net.2.weight"], gn_weight=wt["norm.weight"], gn_bias=wt["norm.bias"],
        wq=wt["graph.query_proj.weight"], bq=wt["graph.query_proj.bias"], wk=wt["graph.key_proj.weight"],
        bk=wt["graph.key_proj.bias"], wm=wt["graph.msg_proj.weight"], bm=wt["graph.msg_proj.bias"],
        scaling=wt["graph.scaling"]))
    offs = roll_offsets(spec)
    d = S.make_desc(B=x.shape[0], C=spec["C"], H=spec["H"], W=spec["H"], hidden=128, d_model=16,
                    offsets=offs[0], flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE,
                    update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                    fire_mode=L.FIRE_HASH, rng_seed=spec["seed"], rng_step=0, sample_base=base)
    out = S.rollout(d, w, x.to(dev).contiguous(), spec["steps"], offs)
    torch.cuda.synchronize()
    plan = (S.k1_variant(d)[0], S.rollout_compact(d), S.rollout_subs(d), S.rollout_fold(d))
    return out, plan


def rollout_rank(rank, world, port, out_path, q):
    import torch
    import torch.distributed as dist

    from graph_neural_cellular_automata_amd.sharding import shard_range
    dev = _init(rank, world, port)
    try:
        spec = ROLL
        x = roll_state(spec)
        s, e = shard_range(spec["B"], rank, world)
        mine, plan = hip_rollout(spec, x[s:e], s, dev)
        mine = mine.cpu()
        bufs = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(bufs, mine)
        plans = [None] * world
        dist.all_gather_object(plans, plan)
        if rank == 0:
            torch.save(torch.cat(bufs), out_path)
            q.put({"plans": plans, "world": dist.get_world_size()})
    except BaseException as exc:   # surface the failure in the parent instead of a silent hang
        q.put({"error": f"rank {rank}: {type(exc).__name__}: {exc}"})
        raise
    finally:
        dist.destroy_process_group()


# ---- the data-parallel training step (train_graph_augmented_nca.py:364-375) --------------------
TRAIN = dict(B=16, C=16, H=40, steps=8, state_seed=55, offset_seed=123, target_seed=99,
             fixture="graph_torus_latest_grown_b1_72")


def train_batch(spec):
    import torch
    g = torch.Generator().manual_seed(spec["state_seed"])
    x = torch.rand(spec["B"], spec["C"], spec["H"], spec["H"], generator=g)
    x[:, 4:] = 0.1 * torch.randn(spec["B"], spec["C"] - 4, spec["H"], spec["H"], generator=g)
    t = torch.rand(4, spec["H"], spec["H"], generator=torch.Generator().manual_seed(spec["target_seed"]))
    t[:3] *= t[3:4]
    return x, t


def train_grads(spec, x, target, dev, policy, max_norm, world_reduce):
    """BPTT through ``steps`` HIP module steps over the batch ``x`` (fire 1.0, message on), the
    trainer's batch-mean premultiplied-RGBA loss, backward, [the flat all-reduce], the policy.
    Returns (averaged grads before the policy, grads after it) as CPU float64 arrays by name."""
    import numpy as np
    import torch

    from graph_neural_cellular_automata_amd import NeuralCAGraph
    from graph_neural_cellular_automata_amd.dp import allreduce_gradients, clip_gradients_, normalize_gradients_
    from graph_neural_cellular_automata_amd.loss import loss_premult_rgba
    from tests.golden_io import Case
    c = Case(spec["fixture"])
    model = NeuralCAGraph(spec["C"], 128, update_gain=0.05, alpha_thr=0.12, message_gain=0.25,
                          graph_zero_padded_shift=False).to(dev)
    model.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in c.weights.items()},
                          strict=False)
    random.seed(spec["offset_seed"])     # every rank draws the same offsets (one random.sample per step)
    state = x.to(dev)
    for _ in range(spec["steps"]):
        state = model(state, fire_rate=1.0)
    loss = loss_premult_rgba(state[:, :4], target.to(dev)[None]).mean()
    params = [p for p in model.parameters() if p.requires_grad]
    loss.backward()
    if world_reduce:
        allreduce_gradients(params)
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    avg = {n: p.grad.detach().double().cpu().numpy() for n, p in zip(names, params) if p.grad is not None}
    if policy == "normalize":
        normalize_gradients_(params)
    else:
        clip_gradients_(params, max_norm)
    post = {n: p.grad.detach().double().cpu().numpy() for n, p in zip(names, params) if p.grad is not None}
    return avg, post


def train_rank(rank, world, port, q, policy, max_norm):
    import torch.distributed as dist

    from graph_neural_cellular_automata_amd.sharding import shard_range
    dev = _init(rank, world, port)
    try:
        x, target = train_batch(TRAIN)
        s, e = shard_range(TRAIN["B"], rank, world)
        avg, post = train_grads(TRAIN, x[s:e], target, dev, policy, max_norm, True)
        if rank == 0:
            q.put({"avg": avg, "post": post})
    except BaseException as exc:
        q.put({"error": f"rank {rank}: {type(exc).__name__}: {exc}"})
        raise
    finally:
        dist.destroy_process_group()


# ---- RCCL on the box: a world_size-1 nccl process group ------------------------
def nccl1_rank(rank, world, port, q):
    """A fresh process (forkserver child: nothing here has touched the GPU before) joins a
    world_size-1 **nccl** (= RCCL) process group and runs the trainer's flat gradient all-reduce
    (``dp.allreduce_gradients``) on the HIP backward's gradients, plus one RCCL sum of a known
    device tensor; the parent compares with its own un-reduced gradients."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        probe = torch.arange(1, 9, dtype=torch.float32, device=dev)
        dist.all_reduce(probe)
        torch.cuda.synchronize()
        x, target = train_batch(TRAIN)
        avg, post = train_grads(TRAIN, x, target, dev, "normalize", 0.0, True)
        q.put({"avg": avg, "post": post, "backend": dist.get_backend(), "world": dist.get_world_size(),
               "probe": probe.cpu().tolist()})
    except BaseException as exc:
        q.put({"error": f"rank {rank}: {type(exc).__name__}: {exc}"})
        raise
    finally:
        dist.destroy_process_group()


def bench_train_nccl(rank, world, port, q, root):
    """``bench.py --mode train --gpus 1 --dist-backend nccl`` for a few iterations, as a child
    process of this forkserver child (which never touches the GPU, so starting a program is safe);
    returns bench's JSON line."""
    import json
    import subprocess
    import sys
    try:
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                   LOCAL_RANK="0")
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--mode", "train", "--gpus", "1",
                            "--dist-backend", "nccl", "--steps", "2", "--warmup", "1"],
                           cwd=root, env=env, capture_output=True, text=True, timeout=100)
        if r.returncode != 0:
            q.put({"error": f"bench rc {r.returncode}: {r.stderr[-2000:]}"})
            return
        q.put({"line": json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])})
    except BaseException as exc:
        q.put({"error": f"{type(exc).__name__}: {exc}"})
        raise


def bench_strong_gloo(rank, world, port, q, root):
    """``bench.py --gpus 2 --scaling strong --dist-backend gloo --batch 256``: bench's own launcher
    starts two ranks on the box's one GPU (a fixed global batch of 256 split 128 per rank, C4's
    fixed-pool form), as a child process of this forkserver child; returns bench's JSON line."""
    import json
    import subprocess
    import sys
    try:
        env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--scaling", "strong",
                            "--dist-backend", "gloo", "--batch", "256", "--steps", "4", "--warmup", "1",
                            "--gpu-warmup-ms", "0", "--no-cpu"],
                           cwd=root, env=env, capture_output=True, text=True, timeout=100)
        if r.returncode != 0:
            q.put({"error": f"bench rc {r.returncode}: {r.stderr[-2000:]}"})
            return
        q.put({"line": json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])})
    except BaseException as exc:
        q.put({"error": f"{type(exc).__name__}: {exc}"})
        raise
