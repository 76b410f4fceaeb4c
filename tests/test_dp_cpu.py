"""world_size-2 gloo check of the data-parallel training step (graph_neural_cellular_automata_amd.dp)
on the CPU: each rank back-propagates the trainer's batch-mean loss over ITS half of the batch
(with the float64 VJP oracle standing in for the GPU backward), the flat-bucket all-reduce
averages the gradients, and the result — before and after the trainer's per-parameter
normalisation — must equal the single-process full-batch gradients."""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nca_oracle as O
from oracle import nca_oracle_vjp as V
from tests.golden_io import Case
from tests.grad_helpers import premult_loss_and_grad

B, H = 4, 12


def _setup(fixture="grad_graph_zeropad_latest_grown_b2_40"):
    c = Case(fixture)
    p = {k: v.astype(np.float64) for k, v in c.weights.items()}
    rng = np.random.default_rng(1)
    x = rng.random((B, 16, H, H))
    x[:, 4:] = rng.standard_normal((B, 12, H, H))
    fire = (rng.random((B, 1, H, H)) < 0.5).astype(np.float64)
    target = rng.random((4, H, H))
    return c, p, x, fire, target


def _grads(lo, hi, fixture="grad_graph_zeropad_latest_grown_b2_40"):
    """Gradients of the mean premultiplied-RGBA loss over samples [lo, hi)."""
    c, p, x, fire, target = _setup(fixture)
    chosen = c.chosen(0) if c.meta["graph"] else None
    out = O.nca_step(x[lo:hi], p, c.cfg(), chosen=chosen, fire_mask=fire[lo:hi])
    _, g = premult_loss_and_grad(out, target)
    _, grads = V.nca_step_vjp(x[lo:hi], p, c.cfg(), g, chosen=chosen, fire_mask=fire[lo:hi])
    return grads


def _params(grads):
    ps = []
    for k in sorted(grads):
        t = torch.zeros(grads[k].shape, dtype=torch.float64, requires_grad=True)
        t.grad = torch.from_numpy(np.array(grads[k], dtype=np.float64))
        ps.append(t)
    return ps


def _worker(rank, world, port, q, fixture=None, policy="normalize"):
    from graph_neural_cellular_automata_amd.dp import POLICIES, allreduce_gradients, clip_gradients_
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    half = B // world
    ps = _params(_grads(rank * half, (rank + 1) * half, *([fixture] if fixture else [])))
    nbytes = allreduce_gradients(ps)
    avg = [p.grad.clone().numpy() for p in ps]
    if policy.startswith("clip:"):   # the classic trainer's clip at a max norm this case exceeds
        clip_gradients_(ps, float(policy[5:]))
    else:
        POLICIES[policy](ps)
    if rank == 0:
        q.put((nbytes, avg, [p.grad.numpy() for p in ps]))
    dist.destroy_process_group()


def _run_two_ranks(fixture=None, policy="normalize"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 1000) + (7 if policy != "normalize" else 0)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, fixture, policy)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    return res


def test_two_rank_allreduce_then_clip_equals_full_batch():
    """The classic trainer's policy (train_intermediate_loss.py:282, clip_grad_norm_) after the
    all-reduce: equals clipping the single-process full-batch gradient (the global norm is not
    linear in the per-rank gradients, so the clip must follow the all-reduce).  This small case's
    gradient norm is ~0.009, so it clips at 0.004 (the trainer's 0.5 would leave it unchanged)."""
    fx, max_norm = "grad_classic_ep980_b2_32", 0.004
    nbytes, avg, clipped = _run_two_ranks(fx, f"clip:{max_norm}")
    full = _grads(0, B, fx)
    keys = sorted(full)
    total = np.sqrt(sum(float((full[k] ** 2).sum()) for k in keys))
    coef = min(1.0, max_norm / (total + 1e-6))
    assert total > max_norm   # the case exercises the clip
    for k, a, c in zip(keys, avg, clipped):
        np.testing.assert_allclose(a, full[k], rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(c, full[k] * coef, rtol=1e-10, atol=1e-15)
    # clipping each rank's gradient before averaging gives a different answer
    halves = [_grads(0, B // 2, fx), _grads(B // 2, B, fx)]
    pre = []
    for h in halves:
        n = np.sqrt(sum(float((h[k] ** 2).sum()) for k in keys))
        pre.append({k: h[k] * min(1.0, max_norm / (n + 1e-6)) for k in keys})
    wrong = {k: 0.5 * (pre[0][k] + pre[1][k]) for k in keys}
    assert max(np.abs(wrong[k] - full[k] * coef).max() for k in keys) > 1e-6


def test_two_rank_allreduce_equals_full_batch():
    nbytes, avg, normed = _run_two_ranks()
    full = _grads(0, B)
    keys = sorted(full)
    assert nbytes == 8 * sum(full[k].size for k in keys)
    for k, a, n in zip(keys, avg, normed):
        np.testing.assert_allclose(a, full[k], rtol=1e-12, atol=1e-15)
        ref = full[k] / (np.linalg.norm(full[k]) + 1e-8)
        np.testing.assert_allclose(n, ref, rtol=1e-10, atol=1e-15)


def test_allreduce_is_noop_without_process_group():
    from graph_neural_cellular_automata_amd.dp import allreduce_gradients
    t = torch.zeros(3, requires_grad=True)
    t.grad = torch.ones(3)
    assert allreduce_gradients([t]) == 0
    assert torch.equal(t.grad, torch.ones(3))
