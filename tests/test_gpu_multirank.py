"""The multi-rank HIP path, test-backed (BASELINE config 4: the pool batch-sharded over GPUs, the
gradient all-reduced before the trainer's normalisation, train_graph_augmented_nca.py:364-375).

Two ranks share the box's one GPU over gloo (fresh forkserver children, tests/mr_workers.py):
  * the sharded rollout (128 samples per rank, C4's per-GPU shard): the all-gathered states equal a
    single-process HIP rollout of the same 256 samples BIT FOR BIT (fire hashed by global sample
    index, per-sample GroupNorm: sharding.py);
  * the data-parallel training step: each rank back-propagates the batch-mean loss of its half of
    the batch through the HIP step, ``dp.allreduce_gradients`` averages the flat bucket, then the
    trainer's policy; the result equals the single-process full-batch gradient after the same
    policy within 1e-6 (``normalize``: the graph trainer's grad/||grad||; ``clip``: the classic
    trainer's clip_grad_norm_, at a max norm the gradient exceeds).
Plus a single-process check that a C4 shard (B=128) rolls out bitwise like the same samples of a
B=1024 rollout."""
import os
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return torch.device("cuda:0")


def _run_ranks(target, args_of_rank, timeout=100):
    import multiprocessing as mp

    assert os.environ.get("GNCA_FORKSERVER_READY") == "1", \
        "the forkserver must start before the GPU is initialised (tests/conftest.py)"
    ctx = mp.get_context("forkserver")
    q = ctx.Queue()
    port = 29900 + (os.getpid() % 500)
    procs = [ctx.Process(target=target, args=(r, 2, port, *args_of_rank(q))) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=timeout)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert "error" not in res, res["error"]
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


def test_two_rank_sharded_rollout_bitwise_equals_one_rank(dev, tmp_path):
    from tests import mr_workers as M
    out = str(tmp_path / "gathered.pt")
    res = _run_ranks(M.rollout_rank, lambda q: (out, q))
    assert res["world"] == 2
    gathered = torch.load(out, weights_only=True)
    spec = M.ROLL
    ref, plan = M.hip_rollout(spec, M.roll_state(spec), 0, dev)
    print(f"[multirank] rollout plans: ranks {res['plans']}, one rank {plan}")
    assert res["plans"][0][0] == "gnca_k1_split<24,36,4,4,8>" and res["plans"][0][1], res["plans"]
    # C4's shard: one stream on the compact field, which folds (round 6); the one-rank reference runs
    # the two-stream pipeline without the fold, so the equality below also crosses the two plans
    assert res["plans"][0][2] == 1 and res["plans"][0][3], "C4's shard: one stream, the compact fold"
    assert torch.equal(gathered, ref.cpu())


@pytest.mark.parametrize("policy", ["normalize", "clip"])
def test_two_rank_dp_gradients_equal_full_batch(dev, policy):
    from tests import mr_workers as M
    spec = M.TRAIN
    x, target = M.train_batch(spec)
    # the full-batch gradient in this process (no all-reduce), and its norm for the clip's bound
    avg_ref, _ = M.train_grads(spec, x, target, dev, "normalize", 0.0, False)
    total = float(np.sqrt(sum((g ** 2).sum() for g in avg_ref.values())))
    max_norm = 0.25 * total            # the clip must act: the case's norm exceeds its bound
    _, post_ref = M.train_grads(spec, x, target, dev, policy, max_norm, False)
    res = _run_ranks(M.train_rank, lambda q: (q, policy, max_norm))
    assert sorted(res["avg"]) == sorted(avg_ref)
    scale = 1.0 / max_norm if policy == "clip" else 1.0   # compare the clipped grads at unit norm
    worst = 0.0
    for k in avg_ref:
        a, r = res["avg"][k], avg_ref[k]
        assert np.abs(a - r).max() <= 1e-6 * max(np.abs(r).max(), 1e-30) + 1e-12, k
        d = np.abs(res["post"][k] - post_ref[k]).max() * scale
        worst = max(worst, d)
        assert d <= 1e-6, (k, d)
    print(f"[multirank] dp {policy}: |grad norm| {total:.3e}, max |2-rank - full batch| after the "
          f"policy (unit scale) {worst:.2e}")


def test_c4_shard_bitwise_equals_full_pool_rollout(dev):
    """BASELINE config 4 on one GPU of eight: a 128-sample shard (sample_base 384) rolls out bitwise
    like the same samples of the whole 1024-sample pool (different plans: the pool runs as two
    sub-batches on two streams, the shard on one)."""
    from tests import mr_workers as M
    spec = dict(M.ROLL, B=1024, steps=6)
    x = M.roll_state(spec)
    full, plan_full = M.hip_rollout(spec, x, 0, dev)
    shard, plan_shard = M.hip_rollout(spec, x[384:512], 384, dev)
    print(f"[multirank] plans: pool {plan_full}, shard {plan_shard}")
    assert plan_full[2] == 2 and not plan_full[3] and plan_shard[2] == 1 and plan_shard[3]
    assert torch.equal(full[384:512], shard)


def _run_one(target, extra=(), timeout=110):
    import multiprocessing as mp

    assert os.environ.get("GNCA_FORKSERVER_READY") == "1", \
        "the forkserver must start before the GPU is initialised (tests/conftest.py)"
    ctx = mp.get_context("forkserver")
    q = ctx.Queue()
    port = 30500 + (os.getpid() % 500)
    p = ctx.Process(target=target, args=(0, 1, port, q, *extra))
    p.start()
    try:
        res = q.get(timeout=timeout)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert "error" not in res, res["error"]
    assert p.exitcode == 0, p.exitcode
    return res


def test_rccl_world1_allreduce_of_hip_gradients(dev):
    """RCCL's own code path on the box (device tensors, its stream ordering, a
    world_size=1 nccl process group): the flat all-reduce of the HIP backward's gradients leaves
    them bit for bit as the un-reduced ones of this process (train_graph_augmented_nca.py:367-375)."""
    from tests import mr_workers as M
    res = _run_one(M.nccl1_rank)
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["probe"] == [float(v) for v in range(1, 9)]
    x, target = M.train_batch(M.TRAIN)
    avg, post = M.train_grads(M.TRAIN, x, target, dev, "normalize", 0.0, False)
    assert sorted(res["avg"]) == sorted(avg)
    for k in avg:
        assert np.array_equal(res["avg"][k], avg[k]), k
        assert np.array_equal(res["post"][k], post[k]), k


def test_rccl_world1_train_bench(dev):
    """``bench.py --mode train --gpus 1 --dist-backend nccl``: the C4/C5 trainer iteration with its
    flat gradient all-reduce through a world-1 RCCL process group."""
    from tests import mr_workers as M
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    line = _run_one(M.bench_train_nccl, (root,), timeout=115)["line"]
    print(f"[multirank] rccl train bench: {line['value']:.3e} cell-upd/s, backend {line['backend']}, "
          f"all-reduce {line['allreduce_bytes']} B")
    assert line["backend"] == "nccl" and line["n_gpus"] == 1
    # one flat fp32 bucket of the parameters that got a gradient (<= the 10,753 trainable ones:
    # gate_mlp never gets one)
    assert 0 < line["allreduce_bytes"] <= 4 * 10753 and line["allreduce_bytes"] % 4 == 0
    assert np.isfinite(line["final_loss"])


def test_bench_strong_scaling_two_ranks_one_gpu(dev):
    """``bench.py --scaling strong --gpus 2``: C4's fixed pool (here 256 samples) split over two ranks
    (both on the box's one GPU, gloo), so the driver's 1 -> 8 GPU run can measure a fixed global batch
    beside the weak-scaling default; the line reports the global batch and each rank's share."""
    from tests import mr_workers as M
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    line = _run_one(M.bench_strong_gloo, (root,), timeout=115)["line"]
    print(f"[multirank] strong-scaling bench, 2 ranks: {line['value']:.3e} cell-upd/s")
    assert line["scaling"] == "strong" and line["n_gpus"] == 2 and line["ranks_seen"] == 2
    assert line["config"]["global_batch"] == 256 and line["config"]["batch_per_gpu"] == 128
    assert len(line["rank_state_checksums"]) == 2 and all(np.isfinite(line["rank_state_checksums"]))
    assert line["value"] == pytest.approx(256 * 72 * 72 * line["steps"] / (line["ms_per_step"] * line["steps"] / 1e3),
                                          rel=1e-6)
