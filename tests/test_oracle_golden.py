"""Pin the CPU oracle (oracle/nca_oracle.py) to the reference's own outputs.

The fixtures were produced by running the reference modules (tests/golden/make_golden.py).
The oracle in float64 must match the reference's float64 run to ~1e-12, and the reference's
float32 run within the reference's intrinsic fp32 noise (1.9e-7 for one step).
"""
import random

import numpy as np
import pytest

from oracle import nca_oracle as O
from tests.golden_io import Case, case_names

CASES = case_names()


def _step(case, x, dtype, t=0):
    p = {k: v.astype(dtype) if v.dtype.kind == "f" else v for k, v in case.weights.items()}
    f = case.fire(t)
    return O.nca_step(x.astype(dtype), p, case.cfg(), chosen=case.chosen(t),
                      fire_mask=None if f is None else f.astype(dtype),
                      return_attention=case.meta["return_attention"])


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_f64(name):
    c = Case(name)
    if not c.has("x_out1_f64"):
        pytest.skip("fixture has no f64 run")
    res = _step(c, c.x_in, np.float64)
    out, attn = res if c.meta["return_attention"] else (res, None)
    np.testing.assert_allclose(out, c.x_out1_f64, rtol=0, atol=1e-6)
    if attn is not None:
        np.testing.assert_allclose(attn, c.attn_f64, rtol=0, atol=1e-5)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_f32(name):
    c = Case(name)
    res = _step(c, c.x_in, np.float32)
    out, attn = res if c.meta["return_attention"] else (res, None)
    np.testing.assert_allclose(out, c.x_out1, rtol=1e-5, atol=2e-6)
    if attn is not None:
        np.testing.assert_allclose(attn, c.attn, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("name", [n for n in CASES if "rollout" in n])
def test_oracle_rollout_matches_reference(name):
    c = Case(name)
    x = c.x_in.astype(np.float64)
    for t in range(c.meta["rollout"]):
        x = _step(c, x, np.float64, t)
    np.testing.assert_allclose(x, c.x_out, rtol=0, atol=1e-4)


def test_offsets_order_matches_reference_sampling():
    """random.sample over the row-major offset list reproduces the recorded draw."""
    for name in CASES:
        c = Case(name)
        if not c.meta["graph"]:
            continue
        offs = O.build_offsets(c.meta["r"])
        k = min(c.meta["K"], len(offs))
        random.seed(c.meta["rng_seed"])
        chosen = random.sample(offs, k) if k > 0 else []
        assert chosen == c.chosen(0), name


def test_offset_counts():
    assert len(O.build_offsets(4)) == 72
    assert len(O.build_offsets(5)) == 112
    assert O.build_offsets(1) == []


def test_pad_shift_ignores_dx():
    z = np.arange(2 * 1 * 5 * 6, dtype=np.float64).reshape(2, 1, 5, 6)
    a = O.shift_pad(z, 2, 3)
    b = O.shift_pad(z, 2, -3)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(a[:, :, 2:], z[:, :, :3])
    assert (a[:, :, :2] == 0).all()


def test_hash_mask_rate_and_shard_invariance():
    m = O.hash_fire_mask(42, 3, 0, 8, 72, 72, 0.5)
    assert abs(m.mean() - 0.5) < 0.01
    part = O.hash_fire_mask(42, 3, 4, 4, 72, 72, 0.5)
    np.testing.assert_array_equal(m[4:], part)
    assert not np.array_equal(O.hash_fire_mask(42, 4, 0, 8, 72, 72, 0.5), m)
