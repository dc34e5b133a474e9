#!/usr/bin/env python3
"""One-GPU measurements of the other BASELINE.json configurations (these are
parity configurations, not the headline bench line): C2 2D 5-pt 4096^2 CG,
C3 3D 7-pt 256^3 CG, C4 conv-diff 256^3 GMRES(30), C5's per-GPU share
(27-pt 512x512x64) CG.  Each: device assembly time, converged solve
(its, reason, time), iterations/s, standalone MatMult time on the bytes the
layout streams (bench.py spmv_format_bytes: x, y, block ids / codes, the
dictionary) as GB/s and fraction of HBM peak, and -- for SURVEY.md §8d's CSR
bytes, which this layout does not move -- the speedup over a CSR SpMV at
peak (not a bandwidth: round 3 printed that figure as "GB/s", up to 105 TB/s)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-petsc4py-example_amd"))
import torch  # noqa: E402

from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import HBM_PEAK_GBS, spmv_bytes, spmv_format_bytes  # noqa: E402

CONFIGS = [("C2", "poisson2d", (4096, 4096, 1), "cg"), ("C3", "poisson3d", (256, 256, 256), "cg"),
           ("C4", "convdiff3d", (256, 256, 256), "gmres"), ("C5/GPU", "poisson3d27", (512, 512, 64), "cg")]


def main():
    comm = DeviceComm.self_comm(0)
    out = []
    for tag, kind, (nx, ny, nz), ksp in CONFIGS:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        A = DMat.stencil(comm, kind, nx, ny, nz)
        torch.cuda.synchronize()
        t_asm = time.perf_counter() - t0
        info = A.info()
        m, nnz = info["m"], info["nnz_d"]
        b = comm.empty(m)
        rhs_hash(comm, 0, b)
        x = comm.zeros(m)
        A.solve(b, x, ksp=ksp, max_it=20, rtol=0.0)      # warm
        x.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = A.solve(b, x, ksp=ksp)
        torch.cuda.synchronize()
        ts = time.perf_counter() - t0
        y = comm.empty(m)
        spmv_ms, _ = A.bench_mult(b, y, 20)
        csr = spmv_bytes(m, nnz, 0)
        streamed = spmv_format_bytes(info, m, nnz, info["nghost"])
        rec = {"config": tag, "kind": kind, "dims": [nx, ny, nz], "ksp": ksp, "rows": m, "nnz": nnz,
               "assembly_s": round(t_asm, 4), "its": r["its"], "reason": r["reason"], "solve_s": round(ts, 4),
               "its_per_s": round(r["its"] / ts, 1), "spmv_ms": round(spmv_ms, 4),
               "spmv_streamed_bytes": streamed, "spmv_GBps": round(streamed / spmv_ms / 1e6, 1),
               "spmv_frac": round(streamed / spmv_ms / 1e6 / HBM_PEAK_GBS, 4),
               "spmv_csr_bytes": csr, "speedup_vs_csr_at_peak": round(csr / (HBM_PEAK_GBS * 1e6) / spmv_ms, 3),
               "dia_slices": info["dia_slices"],
               "pair_shape": info["pair_shape"], "pair_blocks": info["pair_blocks"]}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        A.destroy()
        del b, x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
