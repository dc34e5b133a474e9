#!/usr/bin/env python3
"""createAIJ(csr=...) h2d phase for host arrays of two origins, alternated:
the stencil generator's own output (bench.host_csr_stencil) and np.copy of
it; for each array the share of its mapping backed by transparent huge pages
(/proc/self/smaps AnonHugePages), the suspect for the registration rate."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from mxsolve.core import DeviceComm, DMat, assembly_times  # noqa: E402


def thp(a):
    """(KiB of the mapping holding a's data backed by huge pages, mapping KiB, data offset in page)"""
    addr = a.ctypes.data
    cur = None
    with open("/proc/self/smaps") as fh:
        for line in fh:
            f = line.split()
            if "-" in f[0] and len(f) >= 5 and all(c in "0123456789abcdef-" for c in f[0]):
                lo, hi = (int(x, 16) for x in f[0].split("-"))
                cur = (lo, hi) if lo <= addr < hi else None
            elif cur and f[0] == "AnonHugePages:":
                return int(f[1]), (cur[1] - cur[0]) >> 10, addr & 4095
    return None


comm = DeviceComm.self_comm(0)
n = 256
for rep in range(3):
    g = bench.host_csr_stencil(n, n, n)
    c = tuple(x.copy() for x in g)
    for tag, arr in (("generator", g), ("np.copy", c)):
        A = DMat.from_csr(comm, arr[0].size - 1, arr[0].size - 1, *arr)
        t = assembly_times()
        A.destroy()
        print(f"rep {rep} {tag:9s}: h2d {t['h2d_ms']:.2f} ms = {t['host_bytes'] / t['h2d_ms'] / 1e6:.1f} GB/s; "
              f"THP (huge KiB, map KiB, offset) ip {thp(arr[0])} cols {thp(arr[1])} vals {thp(arr[2])}", flush=True)
    del g, c
