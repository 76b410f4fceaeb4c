"""Data-parallel BPTT training: one flat-bucket gradient all-reduce per optimiser step.

SURVEY.md §8e / §8f rank 1: the graph trainer (``train_graph_augmented_nca.py:362-375``) does

    loss.backward()
    for p in model.parameters():                  # per-parameter grad normalisation
        if p.grad is not None: p.grad.data.div_(p.grad.data.norm().add_(1e-8))
    optimizer.step()

and the classic trainer (``train_intermediate_loss.py:279-283``) clips the global norm instead:

    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 0.5)
    optimizer.step()

Sharded over G GPUs (one process per GPU, each with its own B/G samples of the batch), the
gradient of the batch-mean loss is the AVERAGE of the per-rank gradients, and it must be averaged
BEFORE the (non-linear) normalisation or clip: both depend on the whole batch's gradient.  The
whole model is ~11k fp32 parameters (43 KB), so the all-reduce is latency-bound: one flat bucket, one RCCL call (``backend="nccl"`` is RCCL on ROCm),
over xGMI.  Parameters that never get a gradient (``gate_mlp``, the frozen perception) are left
out — their ``.grad`` stays ``None`` on every rank, because every rank draws the same offsets.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def allreduce_gradients(params, group=None, average: bool = True) -> int:
    """All-reduce (sum, then / world if ``average``) the ``.grad`` of every parameter that has
    one, as ONE flat bucket.  Returns the number of bytes reduced.  No-op when not distributed."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads or not dist.is_available() or not dist.is_initialized():
        return 0
    world = dist.get_world_size(group)
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    if average and world > 1:
        flat.div_(world)
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n
    return flat.numel() * flat.element_size()


def normalize_gradients_(params, eps: float = 1e-8) -> None:
    """The trainers' per-parameter ``grad / (||grad|| + eps)`` (train_graph_augmented_nca.py:371-373).
    Call it after ``allreduce_gradients``."""
    for p in params:
        if p.grad is not None:
            p.grad.div_(p.grad.norm().add_(eps))


def clip_gradients_(params, max_norm: float = 0.5) -> torch.Tensor:
    """The classic trainer's ``clip_grad_norm_(model.parameters(), 0.5)``
    (train_intermediate_loss.py:282): one global 2-norm over every gradient, scale by
    ``max_norm / (norm + 1e-6)`` when that is below 1.  Call it after ``allreduce_gradients``.
    Returns the pre-clip total norm."""
    return torch.nn.utils.clip_grad_norm_([p for p in params if p.grad is not None], max_norm)


# the trainers' gradient policies, applied after the all-reduce
POLICIES = {"normalize": normalize_gradients_,        # train_graph_augmented_nca.py:371-373
            "clip": clip_gradients_}                  # train_intermediate_loss.py:282


def train_step(model, optimizer, loss, group=None, policy: str = "normalize") -> None:
    """backward -> flat all-reduce -> the trainer's gradient policy -> optimizer step.
    ``policy``: "normalize" (graph trainer) or "clip" (classic trainer, max norm 0.5)."""
    optimizer.zero_grad(set_to_none=True)
    loss.backward()
    params = [p for p in model.parameters() if p.requires_grad]
    allreduce_gradients(params, group=group)
    POLICIES[policy](params)
    optimizer.step()
