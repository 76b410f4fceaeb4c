"""BPTT driver for the gradient fixtures: the graph trainer's inner loop
(``train_graph_augmented_nca.py:302-321``) and loss (``:52-61``), written against a pluggable
step + vjp so the same driver runs the CPU oracle and the HIP path."""
from __future__ import annotations

import numpy as np


def premult_loss_and_grad(state: np.ndarray, target: np.ndarray):
    """loss = mean_b mean_{4,H,W} (rgba_premult(state) - target)^2 and d loss / d state."""
    B, C, H, W = state.shape
    a = state[:, 3:4]
    rgb = state[:, :3] * a
    r_rgb = rgb - target[None, :3]
    r_a = a - target[None, 3:4]
    n = 4 * H * W
    loss = float(((r_rgb ** 2).sum() + (r_a ** 2).sum()) / (n * B))
    g = np.zeros_like(state)
    s = 2.0 / (n * B)
    g[:, :3] = s * r_rgb * a
    g[:, 3:4] = s * ((r_rgb * state[:, :3]).sum(1, keepdims=True) + r_a)
    return loss, g


def bptt_oracle(case, step_fn, vjp_fn, dtype=np.float64):
    """Forward the recorded rollout with ``step_fn(x, cfg, chosen, fire)``, then back-propagate
    the trainer's loss with ``vjp_fn(x, cfg, gy, chosen, fire) -> (gx, grads)``."""
    x = case.x_in.astype(dtype)
    T = int(case.meta["rollout"])
    base = case.cfg()
    tape = []
    for t in range(T):
        mask = case.active[t].astype(bool)
        cfg = dict(base, message_gain=base["message_gain"] if case.use_graph[t] else 0.0)
        fire = case.fire_mask[t][mask].astype(dtype) if case.fire_rates[t] < 1.0 else None
        chosen = [tuple(int(v) for v in o) for o in case.offsets[t]]
        sub = x[mask]
        tape.append((sub, mask, cfg, chosen, fire))
        x = x.copy()
        x[mask] = step_fn(sub, cfg, chosen, fire)
    loss, g = premult_loss_and_grad(x, case.target.astype(dtype))
    total = {}
    for sub, mask, cfg, chosen, fire in reversed(tape):
        gx, grads = vjp_fn(sub, cfg, g[mask], chosen, fire)
        g = g.copy()
        g[mask] = gx
        for k, v in grads.items():
            total[k] = total.get(k, 0) + v
    return x, loss, g, total
