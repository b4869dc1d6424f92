import multiprocessing
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Multi-process GPU tests (ranks, the NF binary, bench.py --gpus 2) start their
# processes from a forkserver that is launched HERE, at collection time, before
# any test initialises the GPU: a process that has initialised the GPU must
# never exec another program, and the forkserver's children are forked from a
# process that never touched it.
FORKSERVER = multiprocessing.get_context("forkserver")
try:
    from multiprocessing import forkserver as _fs
    _fs.set_forkserver_preload([])
    _fs.ensure_running()
except (OSError, ValueError):   # pragma: no cover - platform without forkserver
    FORKSERVER = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: full-size (1M-frame) parity runs")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import csum_oracle
    return csum_oracle.load()


@pytest.fixture(scope="session")
def clean_ctx():
    """A multiprocessing context whose processes never inherit a GPU context."""
    if FORKSERVER is None:
        pytest.skip("no forkserver on this platform")
    return FORKSERVER


@pytest.fixture(autouse=True)
def _gpu_fault_attribution(request):
    """After every GPU test: wait for the device, give HIP's event thread a
    moment, and make one more HIP call, so an asynchronously reported fault
    (a GPU memory fault reaches HIP through its event thread, after the kernel
    has ended) fails the test that caused it, not a later one."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import time
    import torch
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
        time.sleep(0.02)
        torch.zeros(1, device="cuda").cpu()
