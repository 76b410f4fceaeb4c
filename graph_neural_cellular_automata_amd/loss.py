"""The graph trainer's loss on the device, fused.

``loss_premult_rgba(pred, target)`` has the reference's signature and result
(``src/training/train_graph_augmented_nca.py:52-61``: full-canvas MSE on premultiplied RGBA,
per-sample [B]); forward and backward are one HIP launch each (``gnca_loss_premult_f32`` /
``gnca_loss_premult_bwd_f32``) instead of the reference's chain of elementwise ops.  ``pred`` may
be the channel slice ``state[:, :4]`` of a contiguous state (read in place through its stride).
"""
from __future__ import annotations

import torch

from . import _lib as L
from .step import stream_ptr


def _strided_ok(t: torch.Tensor) -> bool:
    B, C, H, W = t.shape
    return t.stride(1) == H * W and t.stride(2) == W and t.stride(3) == 1


class _PremultLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target):
        B, _, H, W = pred.shape
        out = torch.empty(B, dtype=torch.float32, device=pred.device)
        tbs = 0 if target.shape[0] == 1 or target.stride(0) == 0 else target.stride(0)
        L.check(L.load().gnca_loss_premult_f32(B, H, W, pred.data_ptr(), pred.stride(0), target.data_ptr(),
                                               tbs, out.data_ptr(), stream_ptr(pred.device)),
                "gnca_loss_premult_f32")
        ctx.save_for_backward(pred, target)
        ctx.tbs = tbs
        return out

    @staticmethod
    def backward(ctx, g):
        pred, target = ctx.saved_tensors
        B, _, H, W = pred.shape
        gp = torch.empty(B, 4, H, W, dtype=torch.float32, device=pred.device)
        g = g.contiguous().float()
        L.check(L.load().gnca_loss_premult_bwd_f32(B, H, W, pred.data_ptr(), pred.stride(0), target.data_ptr(),
                                                   ctx.tbs, g.data_ptr(), gp.data_ptr(), gp.stride(0),
                                                   stream_ptr(pred.device)),
                "gnca_loss_premult_bwd_f32")
        return gp, None


def loss_premult_rgba(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Per-sample [B] MSE between (pred_rgb * pred_alpha, pred_alpha) and target ([B or 1,4,H,W])."""
    if pred.dim() != 4 or pred.shape[1] != 4:
        raise ValueError("pred must be [B,4,H,W]")
    B, _, H, W = pred.shape
    if target.dim() == 3:
        target = target.unsqueeze(0)
    # the kernels index the target with pred's geometry: reject what F.mse_loss could not
    # broadcast (the reference raises there) instead of reading out of bounds on the device
    if target.dim() != 4 or tuple(target.shape[1:]) != (4, H, W) or target.shape[0] not in (1, B):
        raise ValueError(f"target of shape {tuple(target.shape)} does not match pred [{B},4,{H},{W}] "
                         f"(expected [4,{H},{W}], [1,4,{H},{W}] or [{B},4,{H},{W}])")
    if pred.device.type != "cuda" or pred.dtype != torch.float32:
        raise RuntimeError("loss_premult_rgba runs on a float32 ROCm tensor (no CPU path)")
    if not _strided_ok(pred):
        pred = pred.contiguous()
    target = target.to(pred.device, torch.float32)
    if target.shape[0] != 1 and target.stride(0) != 0:
        target = target.contiguous()
    else:
        target = target[:1].contiguous()
    return _PremultLoss.apply(pred, target)
