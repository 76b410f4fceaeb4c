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


def _cfg(cfg: dict, key: str, legacy: str | None, default):
    """``cfg[key]``, else the older key name the reference also accepts, else ``default``."""
    if key in cfg:
        return cfg[key]
    if legacy is not None and legacy in cfg:
        return cfg[legacy]
    return default


# kind -> launcher(state, size, knobs).  ``size`` is the policy's sampled patch size; ``knobs``
# the parsed config (damage.py:118-136 maps each kind to one of the primitives above).
_KINDS = {
    "square": lambda st, n, k: cutout_square_(st, n),
    "circle": lambda st, n, k: cutout_circle_(st, n // 2 if n > 1 else 1),
    "stripes": lambda st, n, k: stripe_wipe_(st, k["stripe_width"], orientation="auto"),
    "alpha_drop": lambda st, n, k: alpha_dropout_(st, k["alpha_dropout_p"], alpha_thr=k["alpha_thr"], hard=True),
    "saltpepper": lambda st, n, k: salt_pepper_alpha_(st, k["salt_pepper_p"]),
    "gaussian": lambda st, n, k: gaussian_hole_(st, radius=max(1, n // 2), softness=k["gaussian_softness"]),
    "hidden_noise": lambda st, n, k: hidden_scramble_(st, sigma=k["hidden_noise_sigma"]),
}


@torch.no_grad()
def apply_damage_policy_(state, dmg_cfg: dict, epoch: int):
    """The reference's policy (damage.py:99-138): from ``start_epoch`` on, with probability
    ``prob`` (one device ``torch.rand(1)``), ONE kind for the whole batch drawn by
    ``random.choices`` over ``kinds``, a patch size by ``random.randint(size_min, size_max)``, then
    that kind's primitive; an unknown kind falls back to the square cut-out.  Same draws, in the
    same order, as the reference."""
    if epoch < int(_cfg(dmg_cfg, "start_epoch", "damage_start_epoch", 100)):
        return
    prob = float(_cfg(dmg_cfg, "prob", "damage_prob", 0.0))
    if prob <= 0 or torch.rand(1, device=state.device).item() > prob:
        return
    table = dmg_cfg.get("kinds", {"square": 1.0})
    kind = random.choices(list(table.keys()), weights=list(table.values()), k=1)[0]
    lo = int(_cfg(dmg_cfg, "size_min", "damage_patch_size", 8))
    size = int(random.randint(lo, int(_cfg(dmg_cfg, "size_max", None, max(lo, 14)))))
    knobs = {"alpha_thr": float(dmg_cfg.get("alpha_thr", 0.1)),
             "alpha_dropout_p": float(dmg_cfg.get("alpha_dropout_p", 0.1)),
             "stripe_width": int(dmg_cfg.get("stripe_width", size)),
             "salt_pepper_p": float(dmg_cfg.get("salt_pepper_p", 0.02)),
             "hidden_noise_sigma": float(dmg_cfg.get("hidden_noise_sigma", 0.0)),
             "gaussian_softness": float(dmg_cfg.get("gaussian_softness", 0.35))}
    _KINDS.get(kind, _KINDS["square"])(state, size, knobs)
