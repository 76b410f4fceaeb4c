"""Pin the backward oracle (oracle/nca_oracle_vjp.py) to the reference's own autograd.

Fixtures: tests/golden/grad_*.npz (one step, seeded cotangent) and bptt_*.npz (the trainer's
masked BPTT loop), made by tests/golden/make_golden_grad.py from the reference modules.
"""
import numpy as np
import pytest

from oracle import nca_oracle as O
from oracle import nca_oracle_vjp as V
from tests.golden_io import Case, bptt_case_names, grad_case_names
from tests.grad_helpers import bptt_oracle

# torus-mode Q/K/scaling grads are exactly 0 in the oracle; the reference's float64 run gives
# ~1e-15 noise (its float32 run ~1e-7) — compared with this absolute floor.
TORUS_ATTN_KEYS = ("graph.scaling", "graph.query_proj", "graph.key_proj")


def _params(case, dtype):
    return {k: v.astype(dtype) if v.dtype.kind == "f" else v for k, v in case.weights.items()}


def assert_grads_close(got: dict, ref: dict, rtol: float, zp: bool, floor: float = 0.0):
    assert set(got) == set(ref), (sorted(got), sorted(ref))
    for k, r in ref.items():
        g = np.asarray(got[k]).reshape(r.shape)
        scale = max(float(np.abs(r).max()), 1e-30)
        if not zp and k.startswith(TORUS_ATTN_KEYS):
            assert float(np.abs(g).max()) <= max(floor, 1e-12), k
            continue
        err = float(np.abs(g - r).max())
        assert err <= rtol * scale + floor, (k, err, scale)


@pytest.mark.parametrize("name", grad_case_names())
def test_vjp_matches_reference_f64(name):
    c = Case(name)
    p = _params(c, np.float64)
    f = c.fire(0)
    gx, grads = V.nca_step_vjp(c.x_in.astype(np.float64), p, c.cfg(), c.cot.astype(np.float64),
                               chosen=c.chosen(0), fire_mask=None if f is None else f.astype(np.float64))
    np.testing.assert_allclose(gx, c.gx_f64, rtol=0, atol=1e-10 * max(1.0, np.abs(c.gx_f64).max()))
    assert_grads_close(grads, c.grads(f64=True), 1e-10, c.meta["zero_padded_shift"])


@pytest.mark.parametrize("name", grad_case_names()[:6])
def test_vjp_forward_consistent(name):
    """The fixture's forward output matches the oracle forward (sanity of the recorded draws)."""
    c = Case(name)
    f = c.fire(0)
    out = O.nca_step(c.x_in.astype(np.float64), _params(c, np.float64), c.cfg(), chosen=c.chosen(0),
                     fire_mask=None if f is None else f.astype(np.float64))
    np.testing.assert_allclose(out, c.x_out1_f64, rtol=0, atol=1e-9)


@pytest.mark.parametrize("name", bptt_case_names())
def test_bptt_oracle_matches_reference(name):
    c = Case(name)
    p = _params(c, np.float64)
    step = lambda x, cfg, ch, f: O.nca_step(x, p, cfg, chosen=ch, fire_mask=f)  # noqa: E731
    vjp = lambda x, cfg, g, ch, f: V.nca_step_vjp(x, p, cfg, g, chosen=ch, fire_mask=f)  # noqa: E731
    x, loss, gx, grads = bptt_oracle(c, step, vjp)
    np.testing.assert_allclose(x, c.x_out_f64, rtol=0, atol=1e-9)
    assert abs(loss - float(c.loss_f64)) <= 1e-12
    np.testing.assert_allclose(gx, c.gx_f64, rtol=0, atol=1e-10 * np.abs(c.gx_f64).max())
    assert_grads_close(grads, c.grads(f64=True), 1e-9, c.meta["zero_padded_shift"])
