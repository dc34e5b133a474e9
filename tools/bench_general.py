#!/usr/bin/env python3
"""Secondary bench legs for the general AIJ path (not the headline line):
matrices that the value-code / code-dictionary compression does not reach.

  varcoef : 3D 7-point variable-coefficient Poisson 256^3, a random face
            coefficient kappa in [1, 2) per interior face -- SPD, ~3 x 256^3
            distinct values, so A_d is stored as fp64 aligned-offset SELL
            (values + one mask byte per row, no column ids);  CG + Jacobi.
  random  : uniform random pattern, 2^24 rows, the diagonal plus 6 columns per
            row drawn uniformly over all 2^24 (test.py's create_system is this
            kind of matrix, scipy.sparse.random), diagonally dominant;
            column-index SELL;  GMRES(30) + Jacobi iterations.
  c4      : BASELINE C4, conv-diff 256^3, GMRES(30) + Jacobi, converged.
  asm     : createAIJ(csr=...) from host int32/fp64 arrays (test.py:24's path)
            by phase -- C3's 256^3 7-point and C5's per-GPU share (27-point
            512 x 512 x 64, 451 M entries); bench.py assembly_from_host.
  (The host baselines of these configurations: python bench.py --cpu-config
   c2|c3|c4|c5share.)

Both general legs go through createAIJ(csr=...) from host arrays
(mx_mat_create_csr), exactly the reference's assembly entry point.  Each leg
prints one JSON line with the MatMult roofline on its streamed bytes (HIP
events around every SpMV launch of a profiled solve, on the library stream)
and on SURVEY.md §8d's CSR bytes.

    python tools/bench_general.py [varcoef|random|c4 ...]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))
import torch  # noqa: E402

from mxsolve.core import DeviceComm, DMat, rhs_hash  # noqa: E402
sys.path.insert(0, ROOT)
from bench import assembly_from_host, spmv_format_bytes  # noqa: E402

PEAK = 8000.0


def varcoef_csr(n: int, seed: int = 7):
    """Natural-ordered 7-point operator with random face coefficients: per row
    the columns -n^2, -n, -1, 0, +1, +n, +n^2 (those inside the grid), off-
    diagonal -kappa(face), diagonal = sum of the 6 face kappas (boundary
    faces kappa = 1, Dirichlet eliminated)."""
    rng = np.random.default_rng(seed)
    N = n ** 3
    i = np.arange(N, dtype=np.int64)
    x, y, z = i % n, (i // n) % n, i // (n * n)
    # kappa of the face between a cell and its +x / +y / +z neighbour
    kx = 1.0 + rng.random(N)
    ky = 1.0 + rng.random(N)
    kz = 1.0 + rng.random(N)
    offs = [-n * n, -n, -1, 0, 1, n, n * n]
    present = [z > 0, y > 0, x > 0, np.ones(N, bool), x < n - 1, y < n - 1, z < n - 1]
    # the face coefficient of each neighbour (the lower cell's kappa)
    kap = [lambda: kz[np.maximum(i - n * n, 0)], lambda: ky[np.maximum(i - n, 0)], lambda: kx[np.maximum(i - 1, 0)],
           None, lambda: kx, lambda: ky, lambda: kz]
    diag = np.zeros(N)
    for j in (0, 1, 2, 4, 5, 6):
        diag += np.where(present[j], kap[j](), 1.0)
    cnt = np.zeros(N, np.int64)
    for p in present:
        cnt += p
    indptr = np.zeros(N + 1, np.int64)
    np.cumsum(cnt, out=indptr[1:])
    nnz = int(indptr[-1])
    cols = np.empty(nnz, np.int32)
    vals = np.empty(nnz, np.float64)
    pos = indptr[:-1].copy()
    for j, o in enumerate(offs):
        sel = np.nonzero(present[j])[0]
        at = pos[sel]
        cols[at] = (sel + o).astype(np.int32)
        vals[at] = diag[sel] if o == 0 else -kap[j]()[sel]
        pos[sel] += 1
    return N, indptr, cols, vals


def random_csr(N: int, k: int = 6, seed: int = 11):
    rng = np.random.default_rng(seed)
    c = rng.integers(0, N, size=(N, k), dtype=np.int64)
    v = -rng.random((N, k))
    rows = np.arange(N, dtype=np.int64)
    cols = np.concatenate([rows[:, None], c], axis=1)
    vals = np.concatenate([(1.0 + np.abs(v).sum(axis=1))[:, None], v], axis=1)
    order = np.argsort(cols, axis=1, kind="stable")
    cols = np.take_along_axis(cols, order, axis=1).astype(np.int32)
    vals = np.take_along_axis(vals, order, axis=1)
    indptr = np.arange(0, N * (k + 1) + 1, k + 1, dtype=np.int64)
    return N, indptr, cols.reshape(-1), vals.reshape(-1)


def streamed_bytes(info) -> int:
    """Bytes the SpMV streams for this layout: value-coded layouts as bench.py
    counts them (codes or dictionary block ids, x once, y once, slice
    metadata); fp64 row pairs (mx_mat_info.pair_f64): K values per row and a
    flag word per 128 rows, x once, y once; other fp64 layouts: A_d slots (aligned-offset slices: 8 B value + the
    row's mask byte; general slices 12 B per slot incl. padding), x read once,
    y written once, 16 B of slice metadata per slice."""
    m, slots = info["m"], info["sell_slots_d"]
    if info.get("pair_f64"):                  # fp64 row pairs: K values per row (0.0 where absent) + a flag word per 128 rows
        return 8 * info["pair_f64"] * m + 4 * (m // 128) + 16 * m
    if info.get("value_codes"):
        return spmv_format_bytes(info, m, info["nnz_d"] + info["nnz_o"], info["nghost"])
    if info["dia_slices"] * 64 >= m:          # every slice aligned-offset
        mat = 8 * slots + m
    else:
        mat = 12 * slots
    return mat + 16 * m + 16 * ((m + 63) // 64)


def gather_bytes(info) -> int:
    """Column-index layouts: each x gather of a random column fetches a whole
    64-byte sector from memory (measured: FETCH_SIZE of the random leg is
    ~64 B per off-diagonal entry, tools/random_spmv.py under rocprofv3), so
    the memory traffic is the slot stream + y + the own-row x (coalesced) +
    64 B per off-diagonal nonzero."""
    m = info["m"]
    return 12 * info["sell_slots_d"] + 16 * m + 16 * ((m + 63) // 64) + 64 * (info["nnz_d"] - m)


def leg(comm, name, A, ksp, rtol=1e-5, max_it=10000, asm_s=None, jac_vec=False):
    """jac_vec: the GMRES MatMult applies a non-uniform Jacobi diagonal to its
    output (SPMV_JACOBI_S), reading the dinv vector: + 8 B per row (not on
    value-coded row pairs, whose dinv comes from the per-code table)."""
    info = A.info()
    m, nnz = info["m"], info["nnz_d"] + info["nnz_o"]
    b = comm.empty(m)
    rhs_hash(comm, 0, b)
    x = comm.zeros(m)
    A.solve(b, x, ksp=ksp, rtol=0.0, max_it=20)               # warm (graph, work space)
    x.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = A.solve(b, x, ksp=ksp, rtol=rtol, max_it=max_it)
    torch.cuda.synchronize()
    ts = time.perf_counter() - t0
    x.zero_()
    rp = A.solve(b, x, ksp=ksp, rtol=0.0, max_it=60, profile=True)
    spmv_ms = rp["spmv_ms"] / max(rp["spmv_count"], 1)
    y = comm.empty(m)
    alone_ms, _ = A.bench_mult(b, y, 30)
    # row-pair layouts with value codes apply Jacobi from the per-code dinv
    # table (dtab, knob 37): no dinv vector is read
    if info.get("value_codes") and info.get("pair_shape"):
        jac_vec = False
    sb = streamed_bytes(info) + (8 * m if jac_vec else 0)
    csr = 12 * nnz + 4 * (m + 1) + 16 * m
    rec = {"leg": name, "rows": m, "nnz": nnz, "ksp": ksp, "value_codes": info["value_codes"],
           "dia_slices": info["dia_slices"], "sell_slots_d": info["sell_slots_d"],
           "assembly_s": None if asm_s is None else round(asm_s, 3),
           "its": r["its"], "reason": r["reason"], "solve_s": round(ts, 4), "its_per_s": round(r["its"] / ts, 1),
           "spmv_in_solve_ms": round(spmv_ms, 5), "spmv_standalone_ms": round(alone_ms, 5),
           "spmv_kernel": ("pair_zmc" if info.get("pair_code") else "pair_zmf64" if info.get("pair_f64")
                           else "pair_lean" if info.get("pair_lean") else "sell"),
           "roofline": {"bound": "hbm", "peak": PEAK, "unit": "GB/s",
                        "streamed_bytes": sb, "achieved": round(sb / spmv_ms / 1e6, 1),
                        "frac": round(sb / spmv_ms / 1e6 / PEAK, 4),
                        "csr_bytes": csr, "csr_achieved": round(csr / spmv_ms / 1e6, 1),
                        "csr_frac": round(csr / spmv_ms / 1e6 / PEAK, 4)}}
    if not info["dia_slices"]:                 # column-index SELL: the gather-aware traffic model
        gb = gather_bytes(info) + (8 * m if jac_vec else 0)
        rec["roofline"].update({"gather_model_bytes": gb, "gather_model_achieved": round(gb / spmv_ms / 1e6, 1),
                                "gather_model_frac": round(gb / spmv_ms / 1e6 / PEAK, 4)})
    print(json.dumps(rec), flush=True)
    del b, x, y
    return rec


def main():
    legs = sys.argv[1:] or ["varcoef", "random", "c4"]
    comm = DeviceComm.self_comm(0)
    for name in legs:
        if name == "varcoef":
            N, ip, c, v = varcoef_csr(256)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            A = DMat.from_csr(comm, N, N, ip, c, v)
            torch.cuda.synchronize()
            asm = time.perf_counter() - t0
            del ip, c, v
            leg(comm, "varcoef 7-pt 256^3 (fp64 values)", A, "cg", asm_s=asm)
        elif name == "random":
            N, ip, c, v = random_csr(1 << 24)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            A = DMat.from_csr(comm, N, N, ip, c, v)
            torch.cuda.synchronize()
            asm = time.perf_counter() - t0
            del ip, c, v
            leg(comm, "random pattern 2^24 rows x 7 (column SELL)", A, "gmres", rtol=0.0, max_it=300, asm_s=asm,
                jac_vec=True)
        elif name == "asm":
            for dims, kind in (((256, 256, 256), "7pt"), ((512, 512, 64), "27pt")):
                print(json.dumps({"leg": "assembly from host CSR", **assembly_from_host(comm, *dims, kind)}), flush=True)
                torch.cuda.empty_cache()
            continue
        elif name == "c4":
            t0 = time.perf_counter()
            A = DMat.stencil(comm, "convdiff3d", 256)
            torch.cuda.synchronize()
            leg(comm, "C4 conv-diff 256^3 GMRES(30)", A, "gmres", asm_s=time.perf_counter() - t0, jac_vec=True)
        A.destroy()
        torch.cuda.empty_cache()
    comm.destroy()


if __name__ == "__main__":
    main()
