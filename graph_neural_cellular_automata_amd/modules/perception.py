"""FixedSobelPerception — mirror of src/modules/perception.py:5-26.

Same constructor, submodule (`conv`) and state_dict key (`perception.conv.weight`); forward runs
the HIP kernel `gnca_perceive` through the C ABI.  Inside the NCA step the perception is fused
into K1 and never materialised.
"""
import torch
import torch.nn as nn

from .. import step as S


class FixedSobelPerception(nn.Module):
    """Frozen depthwise conv: identity + Sobel-x + Sobel-y per channel (perception.py:7-19)."""

    def __init__(self, n_channels):
        super().__init__()
        ident = torch.zeros(3, 3)
        ident[1, 1] = 1.0
        sx = torch.tensor([[1.0, 0.0, -1.0], [2.0, 0.0, -2.0], [1.0, 0.0, -1.0]])
        sy = sx.t().contiguous()  # [[1,2,1],[0,0,0],[-1,-2,-1]]
        bank = torch.stack([ident, sx, sy]).unsqueeze(1)          # [3,1,3,3]
        self.conv = nn.Conv2d(n_channels, 3 * n_channels, 3, 1, 1, groups=n_channels, bias=False)
        with torch.no_grad():
            self.conv.weight.copy_(bank.repeat(n_channels, 1, 1, 1))
        self.conv.weight.requires_grad_(False)

    def forward(self, x):
        """[B,C,H,W] -> [B,3C,H,W] ordered [identity(C), sobel_x(C), sobel_y(C)] (perception.py:25)."""
        x = S.check_state(x, x.shape[1]) if x.shape[1] >= 4 else S._dev_f32(x, "state")
        return S.perceive(self.conv.weight, x)
