"""GraphAugmentation — mirror of src/modules/graph_augmentation.py:8-169.

Same constructor, attributes (num_neighbors, offsets, zero_padded_shift, alive_to_alive,
alpha_thr, scaling, query/key/msg_proj, gate_mlp) and state_dict keys.  forward() draws the
offsets with exactly one ``random.sample`` (graph_augmentation.py:120-121) and runs the HIP
message kernel (K0 + message-only K1) through the C ABI.
"""
import math
import random

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib as L
from .. import step as S


class GraphAugmentation(nn.Module):
    def __init__(self, n_channels: int, d_model: int = 16, attention_radius: int = 4,
                 num_neighbors: int = 8, gating_hidden: int = 32, *, alive_to_alive: bool = True,
                 zero_padded_shift: bool = True, alpha_thr: float = 0.1):
        super().__init__()
        self.n_channels = n_channels
        self.d_model = d_model
        self.attention_radius = attention_radius
        self.num_neighbors = num_neighbors
        self.alive_to_alive = bool(alive_to_alive)
        self.zero_padded_shift = bool(zero_padded_shift)
        self.alpha_thr = float(alpha_thr)
        # same construction order as the reference => same default init under the same seed
        self.query_proj = nn.Conv2d(n_channels, d_model, 1)
        self.key_proj = nn.Conv2d(n_channels, d_model, 1)
        self.msg_proj = nn.Conv2d(n_channels, n_channels, 1)
        self.scaling = nn.Parameter(torch.tensor(math.sqrt(d_model), dtype=torch.float32))
        # never used in forward (the reference's channel gate is dead code, graph_aug.py:62-68);
        # kept so checkpoints load with no missing/unexpected keys
        self.gate_mlp = nn.Sequential(
            nn.Conv2d(n_channels * 2, gating_hidden, 1), nn.ReLU(inplace=False),
            nn.Conv2d(gating_hidden, n_channels, 1), nn.Sigmoid())
        self.offsets = self._build_offsets(attention_radius)

    @staticmethod
    def _build_offsets(radius: int):
        """Row-major (dy, dx) in [-r, r]^2 without the 3x3 block (graph_augmentation.py:73-83)."""
        return [(dy, dx) for dy in range(-radius, radius + 1) for dx in range(-radius, radius + 1)
                if not (abs(dy) <= 1 and abs(dx) <= 1)]

    @staticmethod
    def _shift2d_pad(x: torch.Tensor, dy: int, dx: int) -> torch.Tensor:
        """The reference's zero-padded shift, including its quirk: only rows move
        (graph_augmentation.py:85-92 — the column slice cancels the horizontal pad)."""
        H = x.shape[2]
        out = torch.zeros_like(x)
        lo, hi = max(dy, 0), min(H, H + dy)
        if lo < hi:
            out[:, :, lo:hi] = x[:, :, lo - dy:hi - dy]
        return out

    @staticmethod
    def _shift2d_roll(x: torch.Tensor, dy: int, dx: int) -> torch.Tensor:
        return torch.roll(x, shifts=(dy, dx), dims=(2, 3))

    def _shift(self, x, dy, dx):
        return self._shift2d_pad(x, dy, dx) if self.zero_padded_shift else self._shift2d_roll(x, dy, dx)

    def sample_offsets(self):
        """The step's one Python-RNG draw (graph_augmentation.py:120-121)."""
        k = min(self.num_neighbors, len(self.offsets))
        return random.sample(self.offsets, k) if k > 0 else []

    def flags(self, return_attention: bool) -> int:
        f = L.GRAPH
        if self.alive_to_alive:
            f |= L.ALIVE_TO_ALIVE
        if self.zero_padded_shift:
            f |= L.ZERO_PAD_SHIFT
        if return_attention:
            f |= L.ATTENTION
        return f

    def weight_tensors(self) -> dict:
        return dict(wq=self.query_proj.weight, bq=self.query_proj.bias, wk=self.key_proj.weight,
                    bk=self.key_proj.bias, wm=self.msg_proj.weight, bm=self.msg_proj.bias,
                    scaling=self.scaling)

    def forward(self, x: torch.Tensor, return_attention_map: bool = False):
        """agg_message [B,C,H,W] (+ attention map [B,H,W]) — graph_augmentation.py:104-169."""
        x = S.check_state(x, self.n_channels)
        chosen = self.sample_offsets()
        B, C, H, W = x.shape
        desc = S.make_desc(B=B, C=C, H=H, W=W, hidden=1, d_model=self.d_model, offsets=chosen,
                           flags=self.flags(return_attention_map), update_gain=0.0,
                           alpha_thr=self.alpha_thr, message_gain=1.0, fire_rate=1.0,
                           fire_mode=L.FIRE_NONE)
        w, keep = S.make_weights(self.weight_tensors())
        m, attn = S.message(desc, w, x, want_attention=return_attention_map)
        del keep
        return (m, attn) if return_attention_map else m
