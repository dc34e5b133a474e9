#!/usr/bin/env python3
"""The 256^3 7-point MatMult warm (back to back) and cold (behind a 1 GB
streamed flush, mx_mat_bench_mult_cold), for PMC passes that tell the two
apart by dispatch order (tools/cold_pmc_table.py: a MatMult right after the
flush kernel is a cold one).  Prints the event times.
    python tools/cold_probe.py [n] [iters]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
it = int(sys.argv[2]) if len(sys.argv) > 2 else 5
comm = DeviceComm.self_comm(0)
A = DMat.stencil(comm, "poisson3d", n)
m = A.info()["m"]
b = comm.empty(m); rhs_hash(comm, 0, b)
y = comm.empty(m)
warm, mult = A.bench_mult(b, y, it)
flush = torch.empty(1 << 27, dtype=torch.float64, device=y.device)
ck, cm = A.bench_mult_cold(b, y, flush, it)
print(f"warm kernel {warm * 1e3:.1f} us (MatMult {mult * 1e3:.1f}); cold kernel {ck * 1e3:.1f} us (span {cm * 1e3:.1f})")
A.destroy()
comm.destroy()
