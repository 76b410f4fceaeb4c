import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


# The multi-rank GPU tests (test_gpu_multirank.py) start their ranks as forks of a forkserver that
# is started HERE, before any test touches the GPU: on the GPU pool a process that has initialised
# the GPU must never exec another program, and a forkserver child never execs at all.
def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs through the C-ABI")
    if "not gpu" in (config.getoption("markexpr") or ""):
        return
    import multiprocessing as mp
    import multiprocessing.forkserver as fs

    import torch
    if torch.cuda.device_count() == 0:   # counts devices without initialising HIP
        return
    mp.get_context("forkserver").set_forkserver_preload([])
    fs.ensure_running()
    # an environment flag, not a module global: pytest may import this file under another module name
    # than the tests' `from tests import conftest`
    os.environ["GNCA_FORKSERVER_READY"] = "1"
