import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()
    return oracle


def pytest_sessionstart(session):
    """Start a multiprocessing fork server while this process has not touched a GPU: the
    multi-process GPU tests (tests/test_gpu_dist_gloo.py) fork their ranks from it, so no rank is
    ever exec'ed from a process that has initialised HIP."""
    import multiprocessing as mp
    from multiprocessing import forkserver
    try:
        mp.get_context("forkserver")
        forkserver.ensure_running()
    except Exception:  # pragma: no cover - the GPU test then reports the failure itself
        pass


def forkserver_context():
    import multiprocessing as mp
    return mp.get_context("forkserver")
