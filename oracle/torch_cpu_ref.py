"""PyTorch-CPU restatement of the NCA step — TEST / BENCH INFRASTRUCTURE ONLY.

The CPU baseline BASELINE.md specifies ("a PyTorch-CPU restatement, all physical cores plus 1
thread, configs C1-C4"): the reference's own op sequence on CPU ATen kernels, written fresh from
the reference's behaviour (not a copy), so that ``bench.py``'s ``cpu_baseline`` times what the
reference's CPU path costs on the GPU box's host cores.  Only ``tests/`` and ``bench.py``'s
``cpu_baseline`` leg use it; the product path (``graph_neural_cellular_automata_amd``) never
imports it and has no CPU fallback.

Op sequence per step (reference ``src/modules/ncagraph.py:106-168``, ``nca.py:64-105``):

* perception: grouped 3x3 ``conv2d`` (zero pad), ``[B,C,3,H,W] -> [B,3,C,H,W]`` reorder
  (``perception.py:21-26``);
* update: 1x1 ``conv2d`` 3C->Hd + ReLU + 1x1 ``conv2d`` Hd->C without bias (``ncagraph.py:131``);
* graph (``graph_augmentation.py:104-169``): Q/K/M 1x1 convs, pooled query, alive mask of x,
  per offset ``torch.roll`` of K, M and the mask, pooled logits, temperature softmax over
  offsets, weighted sum; message policy (hidden channels only, tanh * gain, ``ncagraph.py:94-104``);
* ``torch.rand(B,1,H,W) <= fire_rate`` mask (only when fire_rate < 1), pre-update alive mask
  (``max_pool2d`` 3x3, -inf pad), GroupNorm(1, C, eps 1e-3), ``x + tanh(dx) * gain``, post-update
  gate of alpha.

Pinned by the golden fixtures (``tests/test_torch_cpu_ref.py``: the recorded offsets and fire mask
reproduce the reference's fp32 output).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def sobel_bank(C: int, dtype=torch.float32) -> torch.Tensor:
    """[3C,1,3,3]: identity, Sobel-x, Sobel-y per channel (perception.py:9-17)."""
    ident = torch.zeros(3, 3, dtype=dtype)
    ident[1, 1] = 1
    sx = torch.tensor([[1, 0, -1], [2, 0, -2], [1, 0, -1]], dtype=dtype)
    sy = torch.tensor([[1, 2, 1], [0, 0, 0], [-1, -2, -1]], dtype=dtype)
    return torch.stack([ident, sx, sy])[:, None].repeat(C, 1, 1, 1)


def build_offsets(radius: int):
    """Row-major (dy, dx) in [-r, r]^2 minus the 3x3 block (graph_augmentation.py:73-83)."""
    return [(dy, dx) for dy in range(-radius, radius + 1) for dx in range(-radius, radius + 1)
            if not (abs(dy) <= 1 and abs(dx) <= 1)]


def _alive(x, thr):
    return (F.max_pool2d(x[:, 3:4], 3, 1, 1) > thr).to(x.dtype)


class TorchCpuStep:
    """One CA step of NeuralCAGraph / NeuralCA on CPU tensors (reference layouts, fp32)."""

    def __init__(self, params: dict, *, graph: bool, update_gain: float, alpha_thr: float,
                 message_gain: float = 0.25, hidden_only: bool = True, alive_to_alive: bool = True,
                 zero_padded_shift: bool = False, use_groupnorm: bool = True):
        t = {k: torch.as_tensor(v, dtype=torch.float32) for k, v in params.items()}
        self.p = t
        self.C = t["update_net.2.weight"].shape[0]
        self.graph = graph
        self.gain, self.thr, self.mgain = update_gain, alpha_thr, message_gain
        self.hidden_only, self.a2a, self.zp, self.use_gn = hidden_only, alive_to_alive, zero_padded_shift, use_groupnorm

    def _shift(self, z, dy, dx):
        if not self.zp:
            return torch.roll(z, shifts=(dy, dx), dims=(2, 3))      # graph_augmentation.py:94-97
        out = torch.zeros_like(z)                                     # :85-92, dx ignored (quirk)
        H = z.shape[2]
        lo, hi = max(dy, 0), min(H, H + dy)
        if lo < hi:
            out[:, :, lo:hi] = z[:, :, lo - dy:hi - dy]
        return out

    def message(self, x, chosen):
        p = self.p
        Q = F.conv2d(x, p["graph.query_proj.weight"], p["graph.query_proj.bias"])
        K = F.conv2d(x, p["graph.key_proj.weight"], p["graph.key_proj.bias"])
        M = F.conv2d(x, p["graph.msg_proj.weight"], p["graph.msg_proj.bias"])
        if not chosen:
            return torch.zeros_like(M)
        qp = Q.mean(dim=(2, 3))
        A = _alive(x, self.thr) if self.a2a else None
        msgs, logits = [], []
        for dy, dx in chosen:
            Ks = self._shift(K, dy, dx)
            Ms = self._shift(M, dy, dx)
            if A is not None:
                Ms = Ms * self._shift(A, dy, dx)
            logits.append((qp * Ks.mean(dim=(2, 3))).sum(dim=1))
            msgs.append(Ms)
        L = torch.stack(logits, 0)
        L = L - L.max(dim=0, keepdim=True).values
        Wt = torch.softmax(L / (p["graph.scaling"].abs() + 1e-6), dim=0)
        return (torch.stack(msgs, 0) * Wt[:, :, None, None, None]).sum(dim=0)

    @torch.no_grad()
    def __call__(self, x, fire_rate: float = 1.0, chosen=None, fire_mask=None):
        p, C = self.p, self.C
        B, _, H, W = x.shape
        y = F.conv2d(x, p["perception.conv.weight"], padding=1, groups=C)
        y = y.view(B, C, 3, H, W).transpose(1, 2).reshape(B, 3 * C, H, W)
        h = torch.relu(F.conv2d(y, p["update_net.0.weight"], p["update_net.0.bias"]))
        dx = F.conv2d(h, p["update_net.2.weight"])
        if self.graph:
            m = self.message(x, chosen or [])
            if self.hidden_only and C >= 4:
                m = torch.cat([torch.zeros_like(m[:, :4]), m[:, 4:]], dim=1)
            dx = dx + torch.tanh(m) * self.mgain
        if fire_mask is not None:
            dx = dx * fire_mask
        elif fire_rate < 1.0:
            dx = dx * (torch.rand(B, 1, H, W) <= fire_rate).to(x.dtype)
        dx = dx * _alive(x, self.thr)
        if self.use_gn:
            dx = F.group_norm(dx, 1, p["norm.weight"], p["norm.bias"], eps=1e-3)
        xt = x + torch.tanh(dx) * self.gain
        post = _alive(xt, self.thr)
        return torch.cat([xt[:, :3], xt[:, 3:4] * post, xt[:, 4:]], dim=1)
