"""NeuralCA — mirror of src/modules/nca.py:7-105 (classic NCA: the step without the graph term)."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ._stepper import run_step
from .perception import FixedSobelPerception


class NeuralCA(nn.Module):
    def __init__(self, n_channels: int, update_hidden: int = 128, img_size: int = 40,
                 update_gain: float = 0.1, alpha_thr: float = 0.1, use_groupnorm: bool = True,
                 device: str = "cpu"):
        super().__init__()
        self.n_channels = n_channels
        self.img_size = img_size          # stored, unused (as in the reference)
        self.update_gain = update_gain
        self.alpha_thr = alpha_thr
        self.device = device              # stored, unused (as in the reference)
        self.perception = FixedSobelPerception(n_channels)
        self.update_net = nn.Sequential(
            nn.Conv2d(n_channels * 3, update_hidden, kernel_size=1, bias=True),
            nn.ReLU(inplace=False),
            nn.Conv2d(update_hidden, n_channels, kernel_size=1, bias=False))
        nn.init.zeros_(self.update_net[-1].weight)
        self.norm = nn.GroupNorm(1, n_channels, eps=1e-3, affine=True) if use_groupnorm else nn.Identity()

    @torch.no_grad()
    def _alive_mask(self, x: torch.Tensor) -> torch.Tensor:
        """max_pool2d(alpha, 3, 1, 1) > alpha_thr (nca.py:55-62); a helper, not the step."""
        return (F.max_pool2d(x[:, 3:4], kernel_size=3, stride=1, padding=1) > self.alpha_thr).float()

    def forward(self, x: torch.Tensor, fire_rate: float = 1.0, *,
                active: torch.Tensor | None = None) -> torch.Tensor:
        """One CA step on the HIP path (nca.py:64-105).  ``active``: see NeuralCAGraph.forward."""
        out, _ = run_step(self, x, fire_rate, None, None, 0.0, False, False, active=active)
        return out
