"""Pin the PyTorch-CPU restatement (oracle/torch_cpu_ref.py, bench.py's CPU baseline) to the
reference's own fp32 outputs recorded in the golden fixtures (same offsets, same fire mask)."""
import numpy as np
import pytest
import torch

from oracle.torch_cpu_ref import TorchCpuStep, build_offsets
from oracle import nca_oracle as O
from tests.golden_io import Case, case_names

CASES = [n for n in case_names() if not Case(n).meta["return_attention"]]


def _stepper(c):
    m = c.meta
    return TorchCpuStep({k: v for k, v in c.weights.items()}, graph=m["graph"],
                        update_gain=m["update_gain"], alpha_thr=m["alpha_thr"],
                        message_gain=m["message_gain"], hidden_only=m["hidden_only"],
                        alive_to_alive=m["alive_to_alive"], zero_padded_shift=m["zero_padded_shift"],
                        use_groupnorm=m["use_groupnorm"])


@pytest.mark.parametrize("name", CASES)
def test_torch_cpu_step_matches_reference_f32(name):
    c = Case(name)
    step = _stepper(c)
    f = c.fire(0)
    x = torch.from_numpy(c.x_in.astype(np.float32))
    out = step(x, chosen=c.chosen(0) if c.meta["graph"] else None,
               fire_mask=None if f is None else torch.from_numpy(f))
    np.testing.assert_allclose(out.numpy(), c.x_out1, rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("name", [n for n in CASES if "rollout" in n])
def test_torch_cpu_rollout_matches_reference(name):
    c = Case(name)
    step = _stepper(c)
    x = torch.from_numpy(c.x_in.astype(np.float32))
    for t in range(c.meta["rollout"]):
        f = c.fire(t)
        x = step(x, chosen=c.chosen(t), fire_mask=None if f is None else torch.from_numpy(f))
    np.testing.assert_allclose(x.numpy(), c.x_out, rtol=0, atol=1e-4)


def test_offsets_and_sobel_bank():
    assert build_offsets(4) == O.build_offsets(4)
    assert build_offsets(5) == O.build_offsets(5)
