"""bench.py's host-side logic (no GPU): the configuration legs check their
converged counts against the ones the full-size parity tests pin, and the
per-kernel roofline records are computed from event time and bytes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def test_config_counts_match_fullsize_tests():
    import bench
    from test_gpu_fullsize import FULL_COUNTS
    for tag, _kind, _dims, _ksp, expect in bench.BENCH_CONFIGS:
        assert FULL_COUNTS[tag] == expect, tag


def test_kernel_frac_record():
    import bench
    assert bench.kernel_frac("k", 1.0, 0, 100) is None
    r = bench.kernel_frac("k", 2.0, 4, 400_000_000)        # 0.5 ms per launch, 400 MB: 800 GB/s
    assert r["avg_launch_ms"] == 0.5 and r["GBps"] == 800.0 and r["frac"] == 0.1


class _Err(Exception):
    pass


def _fake_lib():
    knobs = {33: 120000, 47: 600000}
    def set_knobs(kn):
        old = {k: knobs.get(k, 0) for k in kn}
        knobs.update(kn)
        return old
    return knobs, set_knobs


def test_leg_budget_sets_deadlines_and_restores():
    """Every leg runs with knobs 33 / 47 at the budget (a leg's own 33 wins),
    and the library's values come back afterwards."""
    import bench
    knobs, set_knobs = _fake_lib()
    seen = []

    def run_leg(name, kn):
        seen.append((name, knobs[33], knobs[47]))
        return {"leg": name, "value": 1.0}
    legs, failed, dead = bench.run_legs([("auto", {}), ("g", {33: 30000})], run_leg, set_knobs, 5.0,
                                        lambda: None, _Err)
    assert [lg["leg"] for lg in legs] == ["auto", "g"] and not failed and dead is None
    assert seen == [("auto", 5000, 5000), ("g", 30000, 5000)]
    assert knobs == {33: 120000, 47: 600000}


def test_leg_budget_watchdog_aborts_a_hung_leg():
    """A leg blocked past twice its budget in a call that polls no deadline is
    aborted by the watchdog (the blocked call then fails): the leg is recorded
    as failed within the budget's bound, later legs do not run, and the legs
    already measured are kept."""
    import threading
    import time
    import bench
    _, set_knobs = _fake_lib()
    aborted = threading.Event()
    ran = []

    def run_leg(name, kn):
        ran.append(name)
        if name == "hung":
            if aborted.wait(20.0):            # a blocked collective, released by the abort
                raise _Err("communicator aborted")
            raise AssertionError("the watchdog never fired")
        return {"leg": name, "value": 2.0}
    t0 = time.perf_counter()
    legs, failed, dead = bench.run_legs([("auto", {}), ("hung", {}), ("later", {})], run_leg, set_knobs, 0.25,
                                        aborted.set, _Err)
    assert time.perf_counter() - t0 < 5.0
    assert ran == ["auto", "hung"] and [lg["leg"] for lg in legs] == ["auto"]
    assert failed[0]["leg"] == "hung" and failed[0]["watchdog_fired"] and "aborted" in dead
    assert 0.4 <= failed[0]["wall_s"] < 5.0


def test_leg_budget_first_leg_failure_raises():
    import bench
    import pytest
    _, set_knobs = _fake_lib()

    def run_leg(name, kn):
        raise _Err("x")
    with pytest.raises(_Err):
        bench.run_legs([("auto", {})], run_leg, set_knobs, 1.0, lambda: None, _Err)


def test_multi_gpu_legs_start_with_the_default():
    """N > 1: the library's default leg runs first, the graph-replay legs last."""
    import re
    src = open(os.path.join(ROOT, "bench.py")).read()
    specs = re.search(r"leg_specs = \[\(\"auto\", \{\}\), (.*?)\]\n", src, re.S).group(1)
    names = re.findall(r"\(\"([^\"]+)\"", specs)
    assert names[-2:] == ["mode2/graph", "mode5/graph"]
    assert bench_parse_stall_ok()


def bench_parse_stall_ok():
    import bench
    return bench.parse_stall("mode2/eager:20") == ("mode2/eager", 20.0) and bench.parse_stall(None) is None
