#!/usr/bin/env python3
"""Interleaved A/B of SpMV variants in one process (methodology: same device,
same data, rounds interleaved).  Prints one JSON line per variant with the
median/min device time per SpMV launch and algorithmic GB/s."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mxsolve import _lib  # noqa: E402
from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "poisson3d"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    L = _lib.load()
    comm = DeviceComm.self_comm(0)
    L.mx_debug_set(4, 0)
    A0 = DMat.stencil(comm, kind, n)          # plain SELL (+ plain copy for A/B)
    L.mx_debug_set(4, 1)
    A1 = DMat.stencil(comm, kind, n)          # aligned-offset slices where they pay
    info = A1.info()
    m, nnz = info["m"], info["nnz_d"]
    alg = 12 * nnz + 4 * (m + 1) + 8 * m + 8 * m
    x = comm.empty(m)
    rhs_hash(comm, 0, x)
    ref = comm.empty(m)
    A0.mult(x, ref)
    variants = {"sell_nt_g8192": (A0, 1, 8192)}
    for g in (1024, 1536, 1792, 2048, 2560, 3584, 4096, 8192):
        variants[f"dia_nt_g{g}"] = (A1, 1, g)
    res = {k: [] for k in variants}
    y = comm.empty(m)
    a = torch.empty(1 << 27, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        b.copy_(a)
    torch.cuda.synchronize()
    copy_gbs = 2 * a.numel() * 8 * 20 / (time.perf_counter() - t0) / 1e9
    del a, b
    for r in range(rounds):
        for k, (A, nt, grid) in variants.items():
            L.mx_debug_set(1, nt); L.mx_debug_set(3, grid)
            y.zero_()
            ms, _ = A.bench_mult(x, y, 20)
            res[k].append(ms)
            if r == 0:
                assert torch.equal(y, ref), k
    L.mx_debug_set(1, 1); L.mx_debug_set(3, 8192)
    print(json.dumps({"kind": kind, "n": n, "rows": m, "nnz": nnz, "alg_bytes": alg,
                      "dia_slices": info["dia_slices"], "slices": (m + 63) // 64,
                      "torch_copy_GBps": round(copy_gbs, 1)}))
    for k, v in res.items():
        med = float(np.median(v))
        print(json.dumps({"variant": k, "median_ms": round(med, 4), "min_ms": round(min(v), 4),
                          "GBps_alg": round(alg / med / 1e6, 1)}))


if __name__ == "__main__":
    main()
