#!/usr/bin/env python3
"""createAIJ(csr=...) from host arrays (bench.py's 256^3 7-point payload,
1.47 GB) three times on fresh arrays and three times on the same arrays:
the host-to-device phase of each (mx_debug_assembly_times)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))
import bench  # noqa: E402
from mxsolve.core import DeviceComm, DMat, assembly_times  # noqa: E402
comm = DeviceComm.self_comm(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
for fresh in (True, True, True, False, False, False):
    if fresh or "ip" not in dir():
        ip, cj, vv = bench.host_csr_stencil(n, n, n)
    A = DMat.from_csr(comm, ip.size - 1, ip.size - 1, ip, cj, vv)
    t = assembly_times()
    print(f"fresh {fresh}: h2d {t['h2d_ms']:.1f} ms = {t['host_bytes'] / t['h2d_ms'] / 1e6:.1f} GB/s, total {t['total_ms']:.1f} ms",
          flush=True)
    A.destroy()
