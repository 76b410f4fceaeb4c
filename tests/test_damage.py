"""Damage ops: the numpy oracle against the reference's outputs (CPU), and
the HIP kernel (gnca_damage_f32) against the same fixtures (GPU).  The fixtures record the
reference's random draws (tests/golden/make_golden_damage.py)."""
import glob
import json
import os

import numpy as np
import pytest
import torch

from oracle.damage_oracle import damage
from tests.golden_io import GOLDEN

NAMES = sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(f"{GOLDEN}/damage_*.npz"))


def _load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files if k != "meta"}, json.loads(str(z["meta"]))


def _oracle(a, m):
    kw = dict(size=m.get("size", 0), pos=a.get("pos"), noise=a.get("noise"), p=m.get("p", 0.0),
              alpha_thr=m.get("alpha_thr", 0.1), hard=m.get("hard", True),
              softness=m.get("softness", 0.35), sigma=m.get("sigma", 0.0),
              orientation=m.get("orientation", "h"))
    return damage(a["x_in"], m["kind"], **kw)


@pytest.mark.parametrize("name", NAMES)
def test_damage_oracle_matches_reference(name):
    a, m = _load(name)
    np.testing.assert_allclose(_oracle(a, m), a["x_out"], rtol=0, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_damage_kernel_matches_reference(name):
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd.damage import _launch
    a, m = _load(name)
    dev = torch.device("cuda:0")
    x = torch.from_numpy(a["x_in"]).to(dev).contiguous()
    kind = {"square": L.DMG_SQUARE, "circle": L.DMG_CIRCLE, "saltpepper": L.DMG_SALT_PEPPER,
            "hidden_noise": L.DMG_HIDDEN_NOISE, "gaussian": L.DMG_GAUSSIAN}.get(m["kind"])
    if m["kind"] == "stripe":
        kind = L.DMG_STRIPE_H if m["orientation"] == "h" else L.DMG_STRIPE_V
    if m["kind"] == "alpha_drop":
        kind = L.DMG_ALPHA_DROP if m["hard"] else L.DMG_ALPHA_DROP_SOFT
    pos = torch.from_numpy(a["pos"]) if "pos" in a else None
    noise = torch.from_numpy(a["noise"]) if "noise" in a else None
    _launch(x, kind, m.get("size", 0), pos=pos, noise=noise, p=m.get("p", 0.0),
            alpha_thr=m.get("alpha_thr", 0.1), softness=m.get("softness", 0.35), sigma=m.get("sigma", 0.0))
    torch.cuda.synchronize()
    np.testing.assert_allclose(x.cpu().numpy(), a["x_out"], rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_damage_policy_api():
    """The reference-named API end to end: shapes and invariants of each kind on the GPU."""
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    from graph_neural_cellular_automata_amd import damage as D
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    x = torch.rand(4, 16, 40, 40, device=dev) + 0.5          # strictly positive
    s = x.clone(); D.cutout_square_(s, 7)
    assert ((s == 0).all(dim=1).flatten(1).sum(1) == 49).all()
    s = x.clone(); D.stripe_wipe_(s, 5, orientation="v")
    assert ((s == 0).all(dim=1).flatten(1).sum(1) == 5 * 40).all()
    s = x.clone(); D.hidden_scramble_(s, 0.2)
    assert torch.equal(s[:, :4], x[:, :4]) and s[:, 4:].max() <= 1.0
    s = x.clone(); D.gaussian_hole_(s, 6)
    assert (s <= x).all() and (s < x * 0.01).any()
    cfg = {"start_epoch": 0, "prob": 1.0, "kinds": {"circle": 1.0}, "size_min": 8, "size_max": 8}
    s = x.clone(); D.apply_damage_policy_(s, cfg, epoch=5)
    assert ((s == 0).all(dim=1).flatten(1).sum(1) > 0).all()
