"""Loader for the golden fixtures written by tests/golden/make_golden.py (data only)."""
from __future__ import annotations

import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _names(pattern):
    return sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(f"{GOLDEN}/{pattern}"))


def case_names():
    """Forward fixtures (make_golden.py)."""
    return [n for n in _names("*.npz") if not n.startswith(("grad_", "bptt_", "damage_"))]


def grad_case_names():
    """One-step gradient fixtures (make_golden_grad.py)."""
    return _names("grad_*.npz")


def bptt_case_names():
    """BPTT rollout gradient fixtures (make_golden_grad.py)."""
    return _names("bptt_*.npz")


class Case:
    def __init__(self, name):
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.name = name
        self.meta = json.loads(str(z["meta"]))
        self.weights = {k[2:]: z[k] for k in z.files if k.startswith("w:")}
        self.arrays = {k: z[k] for k in z.files if not k.startswith("w:") and k != "meta"}

    def __getattr__(self, k):
        try:
            return self.arrays[k]
        except KeyError:
            raise AttributeError(k)

    def has(self, k):
        return k in self.arrays

    def cfg(self):
        m = self.meta
        return dict(update_gain=m["update_gain"], alpha_thr=m["alpha_thr"],
                    use_groupnorm=m["use_groupnorm"], graph=m["graph"],
                    message_gain=m["message_gain"], hidden_only=m["hidden_only"],
                    zero_padded_shift=m["zero_padded_shift"], alive_to_alive=m["alive_to_alive"])

    def grads(self, f64=True):
        """The reference's parameter gradients, keyed like the state_dict."""
        pre = "g64:" if f64 else "g:"
        return {k[len(pre):]: v for k, v in self.arrays.items() if k.startswith(pre)}

    def chosen(self, t=0):
        return [tuple(int(v) for v in o) for o in self.offsets[t]]

    def fire(self, t=0):
        return self.fire_mask[t].astype(np.float32) if self.has("fire_mask") else None
