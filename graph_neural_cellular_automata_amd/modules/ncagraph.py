"""NeuralCAGraph — mirror of src/modules/ncagraph.py:10-168.

Same constructor signature, attributes (message_gain is read per call, alpha_thr, hidden_only,
update_gain), submodules (perception, update_net, norm, graph) and state_dict keys, so the
reference's trainer, test scripts and checkpoints use it unchanged.  forward() keeps the
reference's RNG contract: one ``random.sample`` (inside the graph step) and, only when
fire_rate < 1, one ``torch.rand(B,1,H,W)`` on x.device.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._stepper import run_step
from .graph_augmentation import GraphAugmentation
from .perception import FixedSobelPerception


class NeuralCAGraph(nn.Module):
    def __init__(self, n_channels: int, update_hidden: int = 128, img_size: int = 40,
                 update_gain: float = 0.1, alpha_thr: float = 0.1, use_groupnorm: bool = True, *,
                 message_gain: float = 0.5, hidden_only: bool = True, graph_d_model: int = 16,
                 graph_attention_radius: int = 4, graph_num_neighbors: int = 8,
                 graph_gating_hidden: int = 32, graph_alive_to_alive: bool = True,
                 graph_zero_padded_shift: bool = True, device: str = "cpu"):
        super().__init__()
        self.n_channels = n_channels
        self.img_size = img_size          # stored, unused (as in the reference)
        self.update_gain = float(update_gain)
        self.alpha_thr = float(alpha_thr)
        self.device = device              # stored, unused (as in the reference)
        self.perception = FixedSobelPerception(n_channels)
        self.update_net = nn.Sequential(
            nn.Conv2d(n_channels * 3, update_hidden, kernel_size=1, bias=True),
            nn.ReLU(inplace=False),
            nn.Conv2d(update_hidden, n_channels, kernel_size=1, bias=False))
        nn.init.zeros_(self.update_net[-1].weight)
        self.norm = nn.GroupNorm(1, n_channels, eps=1e-3, affine=True) if use_groupnorm else nn.Identity()
        self.graph = GraphAugmentation(
            n_channels=n_channels, d_model=graph_d_model, attention_radius=graph_attention_radius,
            num_neighbors=graph_num_neighbors, gating_hidden=graph_gating_hidden,
            alive_to_alive=graph_alive_to_alive, zero_padded_shift=graph_zero_padded_shift,
            alpha_thr=self.alpha_thr)
        self.message_gain = float(message_gain)
        self.hidden_only = bool(hidden_only)

    @torch.no_grad()
    def _alive_mask(self, x: torch.Tensor) -> torch.Tensor:
        """max_pool2d(alpha, 3, 1, 1) > alpha_thr (ncagraph.py:85-92); a helper, not the step."""
        return (F.max_pool2d(x[:, 3:4], kernel_size=3, stride=1, padding=1) > self.alpha_thr).float()

    def _apply_message_policy(self, m: torch.Tensor) -> torch.Tensor:
        """hidden_only zeroing + tanh * message_gain (ncagraph.py:94-104); a helper — inside the
        step this is fused into K1's epilogue."""
        if self.hidden_only and m.shape[1] >= 4:
            m = torch.cat([torch.zeros_like(m[:, :4]), m[:, 4:]], dim=1)
        return torch.tanh(m) * self.message_gain

    def forward(self, x: torch.Tensor, fire_rate: float = 1.0, *, return_attention: bool = False,
                active: torch.Tensor | None = None):
        """One CA step with the mid-range graph message, on the HIP path (ncagraph.py:106-168).

        ``active`` (extension, not in the reference): a [B] bool mask; ``model(x, fr, active=m)``
        equals the trainers' ``x[m] = model(x[m], fr)`` (train_graph_augmented_nca.py:305-321)
        without the sub-batch gather/scatter, except that the fire uniforms are drawn for the
        whole batch (``torch.rand(B,1,H,W)``) rather than for the active rows only."""
        chosen = self.graph.sample_offsets()
        out, attn = run_step(self, x, fire_rate, self.graph, chosen, self.message_gain,
                             self.hidden_only, return_attention, active=active)
        return (out, attn) if return_attention else out
