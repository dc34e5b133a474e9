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


def _knobs(L):
    """Every mx_debug_set key's current value (set to a probe value and back:
    a valid key returns the probe value on the way back, an unknown one -1).
    Key 81 is probed with 1, not 0: setting it to 0 empties the device buffer
    cache, and the cache's blocks must carry over from test to test (under
    key 81 = 2 a block read before it is written shows up across tests too)."""
    vals = {}
    for k in range(1, 100):
        probe = 1 if k == 81 else 0
        old = L.mx_debug_set(k, probe)
        if L.mx_debug_set(k, old) == probe:
            vals[k] = old
    return vals


@pytest.fixture(autouse=True)
def _knobs_restored(request):
    """A GPU test leaves the library's knobs as it found them: the knobs are
    process-global, and one left changed silently alters every later test
    (a default path that no longer runs).  A leak is undone and fails the test
    that caused it."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    from mxsolve import _lib
    L = _lib.load()
    before = _knobs(L)
    yield
    after = _knobs(L)
    leaked = {k: (before[k], after.get(k)) for k in before if after.get(k) != before[k]}
    for k, (v, _) in leaked.items():
        L.mx_debug_set(k, v)
    if leaked:
        pytest.fail(f"knobs left changed (key: (before, after)): {leaked}")
