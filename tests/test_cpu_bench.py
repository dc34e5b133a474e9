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
