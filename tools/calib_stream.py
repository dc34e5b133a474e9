#!/usr/bin/env python3
"""FETCH_SIZE calibration: stream 1 GiB (2^27 doubles) once at 8 B and at 16 B
per lane; run under rocprofv3 --pmc FETCH_SIZE to get counter-bytes per
algorithmic byte for each access width (MI355X_MICROARCH.md §HBM: calibrate
before trusting an absolute)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm  # noqa: E402

comm = DeviceComm.self_comm(0)
n = 1 << 27
x = comm.zeros(n)
out = comm.zeros(2048)
for w in (8, 16):
    for _ in range(3):
        _lib.call("mx_debug_stream_read", comm.h, C.c_void_p(x.data_ptr()), n, w, C.c_void_p(out.data_ptr()))
print("streamed", n * 8, "bytes per launch")
