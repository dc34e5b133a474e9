"""Test configuration: paths, the `gpu` marker, shared fixtures."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpi-petsc4py-example_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


_HEARTBEAT_S = float(os.environ.get("MX_TEST_HEARTBEAT_S", "60"))


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_call(item):
    """A test running longer than a minute (the full-size oracle parity runs:
    C2's 7,723 oracle iterations take 2-3 min) prints a line to stderr every
    MX_TEST_HEARTBEAT_S seconds, so a runner that takes a silent process for a
    hung one sees progress."""
    import threading
    import time
    done = threading.Event()

    capman = item.config.pluginmanager.getplugin("capturemanager")

    def beat():
        t0 = time.time()
        while not done.wait(_HEARTBEAT_S):
            msg = f"[still running {item.nodeid}: {time.time() - t0:.0f} s]\n"
            if capman is not None:       # past the output capture, to the real stderr
                with capman.global_and_fixture_disabled():
                    sys.stderr.write(msg)
                    sys.stderr.flush()
            else:
                sys.stderr.write(msg)
                sys.stderr.flush()

    th = threading.Thread(target=beat, daemon=True)
    if _HEARTBEAT_S > 0:
        th.start()
    try:
        yield
    finally:
        done.set()


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "reference_systems.npz")))


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    return oracle


_SELF = []


@pytest.fixture(scope="session")
def selfcomm():
    from mxsolve.core import DeviceComm
    c = DeviceComm.self_comm(0)
    _SELF.append(c)
    yield c


@pytest.fixture(autouse=True)
def _selfcomm_stream():
    """Every test starts with the session communicator's stream as torch's
    current stream: a test that created (and destroyed) another communicator
    made that one current, and torch ops on the session's vectors would
    otherwise be ordered on a different stream than the library's kernels."""
    if _SELF and _SELF[0].h:
        _SELF[0].activate()
    yield
