"""Damage curriculum on the device: the reference's ``utils.damage``
(``src/utils/damage.py:15-138``) with the same function names, arguments and effects, each one
HIP launch over the whole batch (``gnca_damage_f32``).

RNG: ``alpha_dropout_``, ``salt_pepper_alpha_`` and ``hidden_scramble_`` draw exactly what the
reference draws (``torch.rand_like`` / ``torch.randn`` of the same shapes), and ``stripe_wipe_``
/ ``apply_damage_policy_`` consume Python ``random`` as the reference does.  The per-sample
positions of the square / circle / gaussian kinds are drawn for the whole batch in one
``torch.randint`` call on the device instead of one host-synchronising call per sample, so their
values differ from the reference's for the same seed (their ranges are the same).
"""
from __future__ import annotations

import ctypes
import random

import torch

from . import _lib as L
from .step import stream_ptr


def _launch(state, kind, size=0, pos=None, noise=None, p=0.0, alpha_thr=0.1, softness=0.35, sigma=0.0):
    if state.device.type != "cuda" or state.dtype != torch.float32 or not state.is_contiguous():
        raise RuntimeError("damage ops run in place on a contiguous float32 ROCm state (no CPU path)")
    B, C, H, W = state.shape
    d = L.DamageDesc(B=B, C=C, H=H, W=W, kind=kind, size=int(size), p=float(p),
                     alpha_thr=float(alpha_thr), softness=float(softness), sigma=float(sigma))
    pos_t = None if pos is None else pos.to(device=state.device, dtype=torch.int32).contiguous()
    noise_t = None if noise is None else noise.to(device=state.device, dtype=torch.float32).contiguous()
    rc = L.load().gnca_damage_f32(ctypes.byref(d), state.data_ptr(),
                                  None if pos_t is None else pos_t.data_ptr(),
                                  None if noise_t is None else noise_t.data_ptr(), stream_ptr(state.device))
    L.check(rc, "gnca_damage_f32")


def _centres(B, H, W, r, device):
    cy = torch.randint(r, max(r + 1, H - r), (B,), device=device)
    cx = torch.randint(r, max(r + 1, W - r), (B,), device=device)
    return torch.stack([cy, cx], 1)


@torch.no_grad()
def cutout_square_(state, size: int):
    """Zero all channels in a random size x size square per sample (damage.py:15-23)."""
    B, C, H, W = state.shape
    if size <= 0:
        return
    y = torch.randint(0, max(1, H - size + 1), (B,), device=state.device)
    x = torch.randint(0, max(1, W - size + 1), (B,), device=state.device)
    _launch(state, L.DMG_SQUARE, size, pos=torch.stack([y, x], 1))


@torch.no_grad()
def cutout_circle_(state, radius: int):
    """Zero all channels inside a random circle of radius R per sample (damage.py:25-36)."""
    B, C, H, W = state.shape
    if radius <= 0:
        return
    _launch(state, L.DMG_CIRCLE, radius, pos=_centres(B, H, W, radius, state.device))


@torch.no_grad()
def stripe_wipe_(state, width: int, orientation: str = "auto"):
    """Zero one random horizontal or vertical band, shared by the batch (damage.py:38-50)."""
    B, C, H, W = state.shape
    if width <= 0:
        return
    if orientation == "auto":
        orientation = "h" if random.random() < 0.5 else "v"
    if orientation == "h":
        y0 = torch.randint(0, max(1, H - width + 1), (1,), device=state.device)
        pos = torch.stack([y0.expand(B), torch.zeros_like(y0).expand(B)], 1)
        _launch(state, L.DMG_STRIPE_H, width, pos=pos)
    else:
        x0 = torch.randint(0, max(1, W - width + 1), (1,), device=state.device)
        pos = torch.stack([torch.zeros_like(x0).expand(B), x0.expand(B)], 1)
        _launch(state, L.DMG_STRIPE_V, width, pos=pos)


@torch.no_grad()
def alpha_dropout_(state, p: float, alpha_thr: float = 0.1, hard: bool = True):
    """Kill a fraction p of the alive alpha pixels (damage.py:52-65)."""
    if p <= 0:
        return
    u = torch.rand_like(state[:, 3:4])
    _launch(state, L.DMG_ALPHA_DROP if hard else L.DMG_ALPHA_DROP_SOFT, noise=u, p=p, alpha_thr=alpha_thr)


@torch.no_grad()
def salt_pepper_alpha_(state, p: float):
    """Zero alpha at random pixels (damage.py:67-72)."""
    if p <= 0:
        return
    _launch(state, L.DMG_SALT_PEPPER, noise=torch.rand_like(state[:, 3:4]), p=p)


@torch.no_grad()
def hidden_scramble_(state, sigma: float = 0.2):
    """Noise on the hidden channels, clamped to [0, 1] (damage.py:74-80)."""
    B, C, H, W = state.shape
    if C <= 4 or sigma <= 0:
        return
    _launch(state, L.DMG_HIDDEN_NOISE, noise=torch.randn(B, C - 4, H, W, device=state.device), sigma=sigma)


@torch.no_grad()
def gaussian_hole_(state, radius: int, softness: float = 0.35):
    """Multiply all channels by 1 - a soft disk per sample (damage.py:82-97)."""
    B, C, H, W = state.shape
    if radius <= 0:
        return
    _launch(state, L.DMG_GAUSSIAN, radius, pos=_centres(B, H, W, radius, state.device), softness=softness)


@torch.no_grad()
def apply_damage_policy_(state, dmg_cfg: dict, epoch: int):
    """The reference's policy (damage.py:99-138): one sampled kind for the whole batch."""
    start_ep = int(dmg_cfg.get("start_epoch", dmg_cfg.get("damage_start_epoch", 100)))
    prob = float(dmg_cfg.get("prob", dmg_cfg.get("damage_prob", 0.0)))
    if epoch < start_ep or prob <= 0:
        return
    if torch.rand(1, device=state.device).item() > prob:
        return
    kinds = dmg_cfg.get("kinds", {"square": 1.0})
    names, weights = zip(*kinds.items())
    kind = random.choices(names, weights=weights, k=1)[0]
    size_min = int(dmg_cfg.get("size_min", dmg_cfg.get("damage_patch_size", 8)))
    size_max = int(dmg_cfg.get("size_max", max(size_min, 14)))
    size = int(random.randint(size_min, size_max))
    alpha_thr = float(dmg_cfg.get("alpha_thr", 0.1))
    alpha_drop_p = float(dmg_cfg.get("alpha_dropout_p", 0.1))
    stripe_width = int(dmg_cfg.get("stripe_width", size))
    saltpepper_p = float(dmg_cfg.get("salt_pepper_p", 0.02))
    hidden_sigma = float(dmg_cfg.get("hidden_noise_sigma", 0.0))
    gaussian_soft = float(dmg_cfg.get("gaussian_softness", 0.35))
    if kind == "square":
        cutout_square_(state, size)
    elif kind == "circle":
        cutout_circle_(state, size // 2 if size > 1 else 1)
    elif kind == "stripes":
        stripe_wipe_(state, stripe_width, orientation="auto")
    elif kind == "alpha_drop":
        alpha_dropout_(state, alpha_drop_p, alpha_thr=alpha_thr, hard=True)
    elif kind == "saltpepper":
        salt_pepper_alpha_(state, saltpepper_p)
    elif kind == "gaussian":
        gaussian_hole_(state, radius=max(1, size // 2), softness=gaussian_soft)
    elif kind == "hidden_noise":
        hidden_scramble_(state, sigma=hidden_sigma)
    else:
        cutout_square_(state, size)
