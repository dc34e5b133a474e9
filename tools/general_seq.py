#!/usr/bin/env python3
"""bench.py's spmv_general leg after what runs before it in bench.py (the
headline 256^3 operator kept alive with its solves, optionally the host-CSR
assembly leg), to reproduce placement effects on the in-solve time.
    python tools/general_seq.py [pre ...]   (pre: stencil, flush, copy, hostasm; none = leg alone)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

pre = sys.argv[1:]
comm = DeviceComm.self_comm(0)
keep = []
if "stencil" in pre:
    A = DMat.stencil(comm, "poisson3d", 256)
    m = A.info()["m"]
    b = comm.empty(m); rhs_hash(comm, 0, b); x = comm.zeros(m)
    A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=50)
    keep += [A, b, x]
if "flush" in pre:
    f = torch.empty(1 << 26, dtype=torch.float64, device="cuda")
    f.fill_(1.0)
    del f
if "copy" in pre:
    bench.stream_copy_gbps(torch.device("cuda", torch.cuda.current_device()), 1 << 24)
if "hostasm" in pre:
    bench.assembly_from_host(comm, 256, 256, 256)
for rep in range(2):
    g = bench.spmv_general_leg(comm, 256)
    print(pre, rep, "in-solve", g["in_solve_ms"], "standalone", g["standalone_ms"], "frac", g["frac"], flush=True)
