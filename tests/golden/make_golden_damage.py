"""Generate tests/golden/damage_*.npz by running the REFERENCE damage ops (src/utils/damage.py).

Run in the build container only (needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_damage.py

Each fixture: the input state, the kind and its knobs, the random draws the reference made
(replayed from the same seed: per-sample positions, stripe orientation/offset, uniforms or
normals), and the reference's output.  Data only.
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np
import torch

REF = "/root/reference"
sys.path.insert(0, os.path.join(REF, "src"))
sys.dont_write_bytecode = True
from utils import damage as D  # noqa: E402  (reference, src/utils/damage.py)

OUT = os.path.dirname(os.path.abspath(__file__))


def state0(seed, B=3, C=8, H=20, W=22):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, C, H, W, generator=g)
    x[:, 3] = torch.where(x[:, 3] > 0.4, x[:, 3], torch.zeros_like(x[:, 3]))
    return x


def save(name, x, out, meta, **arrays):
    fields = dict(x_in=x.numpy(), x_out=out.numpy(), meta=np.array(json.dumps(meta)))
    fields.update({k: np.asarray(v) for k, v in arrays.items()})
    np.savez_compressed(os.path.join(OUT, f"damage_{name}.npz"), **fields)
    print(name, meta)


def positions(B, lo_hi_y, lo_hi_x):
    pos = []
    for _ in range(B):
        y = int(torch.randint(lo_hi_y[0], lo_hi_y[1], (1,)))
        x = int(torch.randint(lo_hi_x[0], lo_hi_x[1], (1,)))
        pos.append((y, x))
    return np.array(pos, np.int32)


def main():
    x = state0(1)
    B, C, H, W = x.shape
    # square
    size = 6
    torch.manual_seed(10)
    pos = positions(B, (0, max(1, H - size + 1)), (0, max(1, W - size + 1)))
    torch.manual_seed(10)
    out = x.clone(); D.cutout_square_(out, size)
    save("square", x, out, dict(kind="square", size=size), pos=pos)
    # circle
    r = 4
    torch.manual_seed(11)
    pos = positions(B, (r, max(r + 1, H - r)), (r, max(r + 1, W - r)))
    torch.manual_seed(11)
    out = x.clone(); D.cutout_circle_(out, r)
    save("circle", x, out, dict(kind="circle", size=r), pos=pos)
    # stripes (both orientations)
    seen = set()
    for seed in range(12, 40):
        random.seed(seed); torch.manual_seed(seed)
        ori = "h" if random.random() < 0.5 else "v"
        if ori in seen:
            continue
        seen.add(ori)
        width = 5
        lim = H if ori == "h" else W
        off = int(torch.randint(0, max(1, lim - width + 1), (1,)))
        random.seed(seed); torch.manual_seed(seed)
        out = x.clone(); D.stripe_wipe_(out, width, orientation="auto")
        save(f"stripe_{ori}", x, out, dict(kind="stripe", size=width, orientation=ori),
             pos=np.array([[off, 0] if ori == "h" else [0, off]] * B, np.int32))
    # alpha dropout hard / soft
    for hard in (True, False):
        torch.manual_seed(15)
        u = torch.rand_like(x[:, 3:4])
        torch.manual_seed(15)
        out = x.clone(); D.alpha_dropout_(out, 0.3, alpha_thr=0.2, hard=hard)
        save(f"alpha_drop_{'hard' if hard else 'soft'}", x, out,
             dict(kind="alpha_drop", hard=hard, p=0.3, alpha_thr=0.2), noise=u.numpy())
    # salt & pepper
    torch.manual_seed(16)
    u = torch.rand_like(x[:, 3:4])
    torch.manual_seed(16)
    out = x.clone(); D.salt_pepper_alpha_(out, 0.25)
    save("saltpepper", x, out, dict(kind="saltpepper", p=0.25), noise=u.numpy())
    # hidden noise
    torch.manual_seed(17)
    n = torch.randn(B, C - 4, H, W)
    torch.manual_seed(17)
    out = x.clone(); D.hidden_scramble_(out, 0.2)
    save("hidden_noise", x, out, dict(kind="hidden_noise", sigma=0.2), noise=n.numpy())
    # gaussian hole
    r = 5
    torch.manual_seed(18)
    pos = positions(B, (r, max(r + 1, H - r)), (r, max(r + 1, W - r)))
    torch.manual_seed(18)
    out = x.clone(); D.gaussian_hole_(out, r, softness=0.35)
    save("gaussian", x, out, dict(kind="gaussian", size=r, softness=0.35), pos=pos)


if __name__ == "__main__":
    main()
