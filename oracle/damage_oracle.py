"""CPU oracle of the damage ops (src/utils/damage.py:15-97) with explicit random draws —
TEST INFRASTRUCTURE ONLY (same rules as oracle/nca_oracle.py).  Pinned to the reference's own
outputs by tests/test_damage.py (fixtures: tests/golden/make_golden_damage.py)."""
from __future__ import annotations

import numpy as np


def damage(x: np.ndarray, kind: str, *, size=0, pos=None, noise=None, p=0.0, alpha_thr=0.1,
           hard=True, softness=0.35, sigma=0.0, orientation="h") -> np.ndarray:
    out = x.copy()
    B, C, H, W = x.shape
    yy = np.arange(H, dtype=np.float32)[:, None]
    xx = np.arange(W, dtype=np.float32)[None, :]
    if kind == "square":                                   # damage.py:15-23
        for b, (y, x0) in enumerate(pos):
            out[b, :, y:y + size, x0:x0 + size] = 0
    elif kind == "circle":                                 # damage.py:25-36
        for b, (cy, cx) in enumerate(pos):
            m = (yy - cy) ** 2 + (xx - cx) ** 2 <= size ** 2
            out[b][:, m] = 0
    elif kind == "stripe":                                 # damage.py:38-50
        y0, x0 = pos[0]
        if orientation == "h":
            out[:, :, y0:y0 + size, :] = 0
        else:
            out[:, :, :, x0:x0 + size] = 0
    elif kind == "alpha_drop":                             # damage.py:52-65
        a = x[:, 3:4]
        drop = (noise < p).astype(x.dtype) * (a > alpha_thr).astype(x.dtype)
        if hard:
            out = out * (1 - drop)
        else:
            out[:, 3:4] = a * (1 - drop)
    elif kind == "saltpepper":                             # damage.py:67-72
        out[:, 3:4] *= 1 - (noise < p).astype(x.dtype)
    elif kind == "hidden_noise":                           # damage.py:74-80
        out[:, 4:] = np.clip(out[:, 4:] + noise * np.float32(sigma), 0, 1)
    elif kind == "gaussian":                               # damage.py:82-97
        for b, (cy, cx) in enumerate(pos):
            r2 = (yy - cy) ** 2 + (xx - cx) ** 2
            s = np.float32(size * max(1e-6, softness))
            m = np.exp(-(r2 / (np.float32(2.0) * s * s)))
            out[b] *= np.clip(1 - m, 0, 1)
    else:
        raise ValueError(kind)
    return out
