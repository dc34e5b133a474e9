#!/usr/bin/env python3
"""Headline benchmark: CG iterations/s + SpMV HBM GB/s on 3D 7-point Poisson 256^3.

BASELINE.json metric: "CG iters/s + SpMV HBM GB/s (% peak), 3D Poisson 256^3 at
1/2/4/8 GPUs" (config C3).  A step is one global KSPSolve_CG iteration (halo +
SpMV + fused vector passes + 2 reductions) of the Jacobi-preconditioned CG on
the 256^3 system; the matrix and right-hand side are generated and assembled
on the GPUs before timing (synthetic data).  Work per step is
fixed across N (strong scaling): value = K / max-over-ranks(time of K steps).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 256]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

The timed solve runs with rtol = 0 so exactly K iterations execute; the
converged solve (default rtol 1e-5) is reported separately as time-to-solution.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpi-petsc4py-example_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak, MI355X_MICROARCH.md chip table
METRIC = "CG iters/s + SpMV HBM GB/s (% peak), 3D Poisson 256³ at 1/2/4/8 GPUs"


def spmv_bytes(m: int, nnz: int, nghost: int) -> int:
    """Algorithmic bytes of one SpMV on one rank:
    fp64 values + int32 columns, row pointer, x (local + ghosts) read once, y written once."""
    return 12 * nnz + 4 * (m + 1) + 8 * (m + nghost) + 8 * m


def spmv_format_bytes(info: dict, m: int, nnz: int, nghost: int) -> int:
    """Algorithmic bytes of one SpMV in the layout the rank actually streams
    (DESIGN.md §4): with value codes, one code byte per stored slot (8 B/row for
    <= 8 offsets, 32 for 27) instead of 12 B/nnz, x (local + ghosts) read once,
    y written once, 16 B of slice metadata per 64 rows, A_o as 12 B/nnz;
    row-pair units whose code blocks come from the block dictionary stream a
    4-byte block index per 128 rows and the dictionary once instead of their
    codes (uniform-slot dictionaries: 256 B of slot values and lane masks per
    block); without codes, SURVEY.md §8d's CSR bytes."""
    if not info.get("value_codes"):
        return spmv_bytes(m, nnz, nghost)
    codes = info["code_bytes"]
    if info.get("pair_blocks"):
        # uniform-slot blocks are read as 256-byte slot-value/lane-mask records
        blk = 256 if info.get("pair_uniform") else info["pair_block_bytes"]
        codes += (4 - info["pair_block_bytes"]) * info["pair_units"] + info["pair_blocks"] * blk
    return (codes + 8 * (m + nghost) + 8 * m + 16 * ((m + 63) // 64)
            + 12 * info["nnz_o"] + 4 * (m + 1) * (info["nnz_o"] > 0))


def cg_iter_bytes(m: int, nnz: int, nghost: int) -> int:
    """SURVEY.md §8d's "fused minimum" CG iteration: SpMV + 88 B/row of vector traffic."""
    return spmv_bytes(m, nnz, nghost) + 88 * m


def cg_spmv_bytes(m: int, nnz: int, nghost: int) -> int:
    """The CG-fused MatMult (SPMV_CG): the SpMV with p_{i-1} as the operand, plus
    r read, x read + written (deferred x step) and p_i written: 32 B/row."""
    return spmv_bytes(m, nnz, nghost) + 32 * m


def pair_meta_bytes(info: dict, m: int, nnz: int, nghost: int) -> int:
    """The layout's non-vector bytes per product (slice metadata, block ids,
    the dictionary, A_o): spmv_format_bytes minus x read and y written."""
    return spmv_format_bytes(info, m, nnz, nghost) - 8 * (m + nghost) - 8 * m


def cg_iter_bytes_design(info: dict, m: int, nnz: int, nghost: int, mode: int, xb: int = 1) -> int:
    """This design's CG iteration with the uniform Jacobi as a scalar, by the
    fusion mode that ran (knob 9): 0 separate passes, MatMult + 72 B/row (p
    update 24, x/r update 48); 1 MatMult-fused, MatMult + 56 (32 in the
    MatMult, r update 24); 2 x step deferred into the p update, MatMult + 64
    (p/x update 40, r update 24); 5 no product stored: the p update, the p.Ap
    pass (p read: 8 + meta) and the residual update (p read again, r read and
    written: 24 + meta).  The p update streams r and p_{i-1} in and p_i out
    (24 B/row) and, with the x steps batched by B (modes 2/5), every B-th
    launch also the B - 1 older directions and x in and x out: 24 + (8 (B - 1)
    + 16) / B B/row per iteration (B = 1: the 40 of the unbatched step)."""
    pupd = 24 * m + (8 * (xb - 1) + 16) * m // max(xb, 1)
    if mode == 5:
        meta = pair_meta_bytes(info, m, nnz, nghost)
        return pupd + (8 * (m + nghost) + meta) + (8 * (m + nghost) + 16 * m + meta)
    if mode == 2:
        return spmv_format_bytes(info, m, nnz, nghost) + pupd + 24 * m
    return spmv_format_bytes(info, m, nnz, nghost) + {0: 72, 1: 56, 4: 48}.get(mode, 64) * m


def cpu_threads() -> tuple[int, str]:
    """Host threads this process may use: the CPU affinity set, capped by a
    cgroup CPU quota and by OMP_NUM_THREADS when set (the GPU box sets it to
    its per-GPU CPU share; nproc there shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = [f"sched_getaffinity {n}"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
            how.append(f"cgroup cpu.max {q}/{per}")
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
        how.append(f"OMP_NUM_THREADS {omp}")
    return max(1, n), ", ".join(how)


def cpu_baseline(grid: int, threads: int, how: str) -> dict:
    """The oracle's C restatement of PETSc's CG (oracle/petsc_oracle.c) on the
    host cores: the full converged solve of the same system (rtol 1e-5,
    Jacobi), SURVEY.md §8d's timing -- the median of 3 solves after one
    warm-up -- plus the host matrix build, a measured time-to-solution."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    t0 = time.perf_counter()
    ip, c, v = oracle.stencil("poisson3d", grid)
    M = ip.size - 1
    A = oracle.OracleMat.from_csr(M, M, ip, c, v)
    del ip, c, v
    b = oracle.rhs_hash(0, M)
    setup = time.perf_counter() - t0
    A.solve(b, ksp="cg", rtol=0.0, max_it=20, nthreads=threads)      # warm-up: threads, pages
    times, r = [], None
    for _ in range(3):
        t0 = time.perf_counter()
        r = A.solve(b, ksp="cg", pc="jacobi", nthreads=threads)    # converged, default tolerances
        times.append(time.perf_counter() - t0)
    dt = sorted(times)[1]
    model = "unknown CPU"
    try:
        with open("/proc/cpuinfo") as f:
            model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"_oracle": {"x": r["x"], "its": int(r["its"]), "reason": int(r["reason"]), "P": 1,
                        "solve_s": round(dt, 3)},
            "value": round(r["its"] / dt, 3), "unit": "CG iterations/s", "cores": threads,
            "kind": "port", "its": int(r["its"]), "reason": int(r["reason"]),
            "solve_s": round(dt, 3), "solve_s_all": [round(t, 3) for t in times], "assembly_s": round(setup, 3),
            "time_to_solution_s": round(dt + setup, 3), "threads_from": how,
            "sample": f"the full converged CG+Jacobi solve ({r['its']} its, rtol 1e-5) of the {grid}^3 7-point "
                      f"system, median of 3 solves after a 20-iteration warm-up, matrix built and assembled on the "
                      f"host first (oracle/petsc_oracle.c, PETSc-restatement not PETSc, 1 rank x {threads} OpenMP "
                      f"threads on {model}, nproc {os.cpu_count()}, solve {dt:.1f} s, build {setup:.1f} s)"}


HOST_LINK_PEAK_GBS = 64.0   # PCIe 5.0 x16, one direction (the MI355X host link)


def host_csr_stencil(nx: int, ny: int, nz: int, kind: str = "7pt"):
    """test.py's input form for createAIJ(csr=...): host numpy arrays, int32
    row pointer and columns (petsc4py's default 32-bit PetscInt), fp64 values,
    rows in natural order, columns ascending -- the 3D 7-point (diag 6, off -1)
    or 27-point (diag 26, off -1) operator of SURVEY.md §8d, built here with
    numpy (no oracle code)."""
    import numpy as np
    M = nx * ny * nz
    r = np.arange(M, dtype=np.int64)
    i, j, k = r % nx, (r // nx) % ny, r // (nx * ny)
    if kind == "7pt":
        offs = [(0, 0, -1), (0, -1, 0), (-1, 0, 0), (0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1)]
        centre = 6.0
    else:
        offs = [(di, dj, dk) for dk in (-1, 0, 1) for dj in (-1, 0, 1) for di in (-1, 0, 1)]
        centre = 26.0
    cols = np.empty((M, len(offs)), dtype=np.int32)
    keep = np.empty((M, len(offs)), dtype=bool)
    for q, (di, dj, dk) in enumerate(offs):
        ok = (i + di >= 0) & (i + di < nx) & (j + dj >= 0) & (j + dj < ny) & (k + dk >= 0) & (k + dk < nz)
        keep[:, q] = ok
        cols[:, q] = (r + di + nx * (dj + ny * dk)).astype(np.int32)
    del i, j, k
    vals = np.where(np.array([o == (0, 0, 0) for o in offs])[None, :], centre, -1.0)
    vals = np.broadcast_to(vals, cols.shape)
    indptr = np.zeros(M + 1, dtype=np.int32)
    np.cumsum(keep.sum(axis=1, dtype=np.int32), out=indptr[1:])
    return indptr, cols[keep], np.ascontiguousarray(vals[keep])


def assembly_from_host(comm, nx: int, ny: int, nz: int, kind: str = "7pt") -> dict:
    """createAIJ(size, csr=(I, J, V)) from host arrays -- the path test.py:24 /
    petsc_funcs.py:6 take -- timed end to end and by phase (host-to-device
    copy, row canonicalisation, MPIAIJ split, SpMV layouts), each phase's
    GB/s on its byte model against the host link or HBM peak."""
    from mxsolve.core import DMat, assembly_times
    import torch
    ip, cj, vv = host_csr_stencil(nx, ny, nz, kind)
    M, nnz = ip.size - 1, int(cj.size)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    A = DMat.from_csr(comm, M, M, ip, cj, vv)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ph = assembly_times()
    info = A.info()
    A.destroy()
    del ip, cj, vv
    canon_b = 4 * nnz + 24 * M           # fused count pass: rowptr + int32 cols read, A_d / A_o counts written
    split_b = 24 * nnz + 32 * M          # fused fill pass: rowptr, cols, vals, split row pointers -> int32 cols, vals, diag
    gbs = lambda b, ms: round(b / (ms * 1e-3) / 1e9, 1) if ms > 0 else None
    return {"workload": f"{kind} {nx}x{ny}x{nz}, int32 I/J + fp64 V host arrays", "rows": M, "nnz": nnz,
            "wall_s": round(wall, 4), "phases_ms": {k: round(v, 3) for k, v in ph.items() if k.endswith("_ms")},
            "host_bytes": int(ph["host_bytes"]),
            "h2d_GBps": gbs(ph["host_bytes"], ph["h2d_ms"]), "host_link_peak_GBps": HOST_LINK_PEAK_GBS,
            "h2d_frac": round(ph["host_bytes"] / (ph["h2d_ms"] * 1e-3) / 1e9 / HOST_LINK_PEAK_GBS, 4)
            if ph["h2d_ms"] > 0 else None,
            "canon_bytes": canon_b, "canon_GBps": gbs(canon_b, ph["canon_ms"]),
            "split_bytes": split_b, "split_GBps": gbs(split_b, ph["split_ms"]),
            "hbm_peak_GBps": HBM_PEAK_GBS, "nnz_d": info["nnz_d"], "pair_shape": info["pair_shape"]}


CPU_CONFIGS = {   # BASELINE.json configurations for the host leg beside the GPU numbers
    "c2": ("poisson2d", (4096, 4096, 1), "cg", 300),
    "c3": ("poisson3d", (256, 256, 256), "cg", 200),
    "c4": ("convdiff3d", (256, 256, 256), "gmres", 120),
    "c5share": ("poisson3d27", (512, 512, 64), "cg", 60),
}


def cpu_baseline_config(name: str, threads: int, how: str) -> dict:
    """The oracle's C restatement (PETSc-restatement, not PETSc) on the host
    cores for another BASELINE configuration: a bounded sample of `its`
    iterations at rtol = 0 (GMRES: whole restart cycles of 30), the median of 3
    after a warm-up, reported as iterations/s -- the host figure the GPU's
    tools/bench_configs.py / tools/bench_general.py numbers stand beside."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    kind, dims, ksp, its = CPU_CONFIGS[name]
    t0 = time.perf_counter()
    ip, c, v = oracle.stencil(kind, *dims)
    M = ip.size - 1
    A = oracle.OracleMat.from_csr(M, M, ip, c, v)
    del ip, c, v
    b = oracle.rhs_hash(0, M)
    setup = time.perf_counter() - t0
    A.solve(b, ksp=ksp, rtol=0.0, max_it=10, nthreads=threads)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        r = A.solve(b, ksp=ksp, pc="jacobi", rtol=0.0, max_it=its, nthreads=threads)
        times.append(time.perf_counter() - t0)
    dt = sorted(times)[1]
    return {"config": name, "kind": kind, "dims": list(dims), "ksp": ksp + ("(30)" if ksp == "gmres" else ""),
            "value": round(r["its"] / dt, 3), "unit": "iterations/s", "cores": threads, "threads_from": how,
            "cpu_kind": "port", "sample": f"{r['its']} iterations at rtol 0, median of 3 after a warm-up "
            f"(oracle/petsc_oracle.c, PETSc-restatement not PETSc), host build {setup:.1f} s",
            "solve_s_all": [round(t, 3) for t in times]}


def stream_copy_gbps(device, n: int) -> float:
    """torch's own device copy of an n-double vector (read + write), the
    same process's HBM reference rate for the numbers above."""
    import torch
    a = torch.empty(n, dtype=torch.float64, device=device).fill_(1.0)
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    return 2 * 8 * n * 20 / (e0.elapsed_time(e1) * 1e-3) / 1e9


def load_traffic(grid: int, n_gpus: int, mode: int, suffix: str | None = None):
    """Committed PMC traffic of the roofline kernel (profiles/spmv_traffic.json,
    key "<grid>^3/N<n>" plus "/mode5" for mode 5's residual update, or the
    given suffix: "/pb" for the direction update)."""
    path = os.path.join(ROOT, "profiles", "spmv_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        key = f"{grid}^3/N{n_gpus}" + (suffix if suffix is not None else "/mode5" if mode == 5 else "")
        return d.get(key)
    except (OSError, ValueError):
        return None


def varcoef_csr(n: int, seed: int = 7):
    """The variable-coefficient 3D 7-point operator of the general-AIJ leg, as
    test.py:24 hands a matrix to createAIJ(csr=...): host int64 row pointer,
    int32 columns (ascending per row, natural ordering), fp64 values.  Face
    coefficient kappa in [1, 2) drawn per face (seed 7), off-diagonal -kappa,
    diagonal = the sum of the six face kappas (boundary faces 1, Dirichlet
    eliminated): SPD with ~3 n^3 distinct values, so the values must be
    streamed (no value codes) -- the fp64 row-pair z-march."""
    import numpy as np
    rng = np.random.default_rng(seed)
    N = n ** 3
    i = np.arange(N, dtype=np.int64)
    x, y, z = i % n, (i // n) % n, i // (n * n)
    kx, ky, kz = 1.0 + rng.random(N), 1.0 + rng.random(N), 1.0 + rng.random(N)
    offs = [-n * n, -n, -1, 0, 1, n, n * n]
    present = [z > 0, y > 0, x > 0, np.ones(N, bool), x < n - 1, y < n - 1, z < n - 1]
    del x, y, z
    kap = [lambda: kz[np.maximum(i - n * n, 0)], lambda: ky[np.maximum(i - n, 0)], lambda: kx[np.maximum(i - 1, 0)],
           None, lambda: kx, lambda: ky, lambda: kz]
    diag = np.zeros(N)
    for j in (0, 1, 2, 4, 5, 6):
        diag += np.where(present[j], kap[j](), 1.0)
    cnt = np.zeros(N, np.int64)
    for q in present:
        cnt += q
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


def csr_rowsum_reference(indptr, cols, vals, x):
    """y = A x summed the way MatMult_SeqAIJ does (PETSc's loop, SURVEY.md §8a
    A7): each row from +0.0, its entries in ascending column order, one
    rounding per multiply and per add (numpy: no contraction).  A checker for
    bit-exactness, built from the caller's own CSR -- not the oracle."""
    import numpy as np
    m = indptr.size - 1
    ln = np.diff(indptr)
    y = np.zeros(m)
    start = indptr[:-1]
    for k in range(int(ln.max()) if m else 0):
        rows = np.nonzero(ln > k)[0]
        at = start[rows] + k
        y[rows] = y[rows] + vals[at] * x[cols[at]]
    return y


def spmv_general_leg(comm, n: int) -> dict:
    """A MatMult whose values must be streamed: the
    variable-coefficient 7-point n^3 operator through createAIJ(csr=...) from
    host int64/int32/fp64 arrays (test.py:24, petsc_funcs.py:6).  MatMult
    checked bit for bit against the row-ordered product of the same CSR; the
    CG + Jacobi solve converged (true residual reported); the MatMult timed
    inside a profiled CG solve (HIP events attached to the kernel's dispatch)
    and standalone, each on the bytes the layout streams (fp64 row pairs: K
    values per row + a flag word per 128 rows, x once, y once) and on SURVEY.md
    §8d's CSR bytes."""
    import numpy as np
    import torch
    from mxsolve.core import DMat, rhs_hash, vnorm, vaxpy
    t0 = time.perf_counter()
    N, ip, cj, vv = varcoef_csr(n)
    t_gen = time.perf_counter() - t0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    A = DMat.from_csr(comm, N, N, ip, cj, vv)
    torch.cuda.synchronize()
    t_asm = time.perf_counter() - t0
    info = A.info()
    m, nnz = info["m"], info["nnz_d"] + info["nnz_o"]
    xh = np.random.default_rng(3).standard_normal(N)
    xt = torch.from_numpy(xh).to(f"cuda:{torch.cuda.current_device()}")
    y = comm.empty(m)
    A.mult(xt, y)
    yref = csr_rowsum_reference(ip, cj, vv, xh)
    bitexact = bool(np.array_equal(y.cpu().numpy().view(np.uint64), yref.view(np.uint64)))
    del ip, cj, vv, yref, xh
    b = comm.empty(m)
    rhs_hash(comm, 0, b)
    x = comm.zeros(m)
    A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=20)        # KSPSetUp, PCSetUp, graph
    x.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = A.solve(b, x, ksp="cg", pc="jacobi")
    torch.cuda.synchronize()
    ts = time.perf_counter() - t0
    A.mult(x, y)                                                      # true residual b - A x
    vaxpy(comm, -1.0, b, y)
    true_rel = vnorm(comm, y) / vnorm(comm, b)
    x.zero_()
    rp = A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=100, profile=1)
    in_ms = rp["spmv_ms"] / max(rp["spmv_count"], 1)
    alone_ms, _ = A.bench_mult(b, y, 50)
    K = info.get("pair_f64") or 0
    streamed = (8 * K * m + 4 * (m // 128) + 16 * m) if K else None
    csr = spmv_bytes(m, nnz, info["nghost"])
    gbs = lambda nb, ms: round(nb / (ms * 1e-3) / 1e9, 1)
    traffic = None
    try:
        with open(os.path.join(ROOT, "profiles", "spmv_traffic.json")) as f:
            traffic = json.load(f).get(f"varcoef{n}^3/N1")
    except (OSError, ValueError):
        pass
    out = {"workload": f"variable-coefficient 7-point {n}^3 (random face kappa, {K and 'fp64 row pairs'}), "
                       "createAIJ(csr=...) from host int64/int32/fp64 arrays, CG + Jacobi",
           "rows": m, "nnz": nnz, "value_codes": info["value_codes"], "pair_f64": K,
           "kernel": "spmv_pair_zmf64_kernel<SPMV_DOT> (CG MatMult: y = A p and p.y, fp64 values streamed)",
           "csr_gen_s": round(t_gen, 2), "assembly_s": round(t_asm, 4),
           "matmult_bitexact_vs_rowsum": bitexact,
           "its": r["its"], "reason": r["reason"], "cg_mode": rp["cg_mode"], "its_per_s": round(r["its"] / ts, 1),
           "true_rel_residual": float(f"{true_rel:.3e}"),
           "in_solve_ms": round(in_ms, 5), "standalone_ms": round(alone_ms, 5),
           "streamed_bytes": streamed, "csr_bytes": csr, "peak": HBM_PEAK_GBS,
           "achieved": gbs(streamed, in_ms) if streamed else None,
           "frac": round(streamed / (in_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if streamed else None,
           "standalone_GBps": gbs(streamed, alone_ms) if streamed else None,
           "standalone_frac": round(streamed / (alone_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if streamed else None,
           "csr_GBps": gbs(csr, in_ms), "csr_frac": round(csr / (in_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "traffic": traffic["bytes_per_launch"] if traffic else None,
           "traffic_source": traffic.get("source") if traffic else None}
    A.destroy()
    del b, x, y, xt
    return out


def random_csr(N: int, k: int = 6, seed: int = 11):
    """test.py:14's matrix family at scale: each row holds its diagonal and k
    off-diagonal columns drawn uniformly over all N (redrawn until no row
    repeats a column, so the CSR is already canonical), columns ascending,
    values -U[0, 1) off the diagonal and 1 + sum |a_ij| on it; host int64 row
    pointer, int32 columns, fp64 values (createAIJ(csr=...), test.py:24)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    rows = np.arange(N, dtype=np.int64)
    c = rng.integers(0, N, size=(N, k), dtype=np.int64)
    while True:
        cols = np.concatenate([rows[:, None], c], axis=1)
        cols.sort(axis=1)
        dup = np.nonzero(np.any(cols[:, 1:] == cols[:, :-1], axis=1))[0]
        if dup.size == 0:
            break
        c[dup] = rng.integers(0, N, size=(dup.size, k), dtype=np.int64)
    del cols
    v = -rng.random((N, k))
    allc = np.concatenate([rows[:, None], c], axis=1)
    allv = np.concatenate([(1.0 + np.abs(v).sum(axis=1))[:, None], v], axis=1)
    del c, v
    order = np.argsort(allc, axis=1, kind="stable")
    cols = np.take_along_axis(allc, order, axis=1).astype(np.int32).reshape(-1)
    vals = np.take_along_axis(allv, order, axis=1).reshape(-1)
    indptr = np.arange(0, N * (k + 1) + 1, k + 1, dtype=np.int64)
    return indptr, cols, vals


def spmv_random_leg(comm, lg: int = 24) -> dict:
    """The unstructured AIJ MatMult: test.py:14's
    random-pattern family at 2^lg rows x 7 through createAIJ(csr=...) from host
    arrays.  MatMult checked bit for bit against the row-ordered product of the
    same CSR (PETSc's MatMult_SeqAIJ order), then timed standalone (warm) and
    cold (behind a 1 GB streamed flush), each against two byte models: the
    streamed bytes (the layout's slots + x once + y once) and the sector model
    (+ one 64-B sector per off-diagonal gather: x's uniformly random reads
    share no line)."""
    import numpy as np
    import torch
    from mxsolve.core import DMat, dispatch_counts
    N = 1 << lg
    t0 = time.perf_counter()
    ip, cj, vv = random_csr(N)
    t_gen = time.perf_counter() - t0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    A = DMat.from_csr(comm, N, N, ip, cj, vv)
    torch.cuda.synchronize()
    t_asm = time.perf_counter() - t0
    info = A.info()
    m, nnz = info["m"], info["nnz_d"] + info["nnz_o"]
    xh = np.random.default_rng(5).standard_normal(N)
    xt = torch.from_numpy(xh).to(f"cuda:{torch.cuda.current_device()}")
    y = comm.empty(m)
    dispatch_counts(reset=True)
    A.mult(xt, y)
    kinds = [k for k, v in dispatch_counts().items() if v]
    yref = csr_rowsum_reference(ip, cj, vv, xh)
    bitexact = bool(np.array_equal(y.cpu().numpy().view(np.uint64), yref.view(np.uint64)))
    del yref, xh
    warm_ms, _ = A.bench_mult(xt, y, 50)
    flush = torch.empty(1 << 27, dtype=torch.float64, device=y.device)
    cold_kernel_ms, cold_ms = A.bench_mult_cold(xt, y, flush, 5)
    del flush
    slots = info["sell_slots_d"]
    streamed = 12 * slots + 16 * m + 16 * ((m + 63) // 64)
    gathers = nnz - m                                  # the off-diagonal entries
    sector = streamed - 8 * m + 64 * gathers           # x read by sectors instead of once
    f = lambda b, ms: round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    g = lambda b, ms: round(b / (ms * 1e-3) / 1e9, 1)
    traffic = None
    try:
        with open(os.path.join(ROOT, "profiles", "spmv_traffic.json")) as fh:
            traffic = json.load(fh).get(f"random2^{lg}/N1")
    except (OSError, ValueError):
        pass
    out = {"workload": f"uniform random pattern, 2^{lg} rows x 7 (diagonal + 6 random columns), createAIJ(csr=...) "
                       "from host int64/int32/fp64 arrays",
           "rows": m, "nnz": nnz, "sell_slots": slots, "kernels": kinds,
           "csr_gen_s": round(t_gen, 2), "assembly_s": round(t_asm, 4),
           "matmult_bitexact_vs_rowsum": bitexact,
           "streamed_bytes": streamed, "sector_bytes": sector, "peak": HBM_PEAK_GBS,
           "warm_ms": round(warm_ms, 5), "warm_GBps_streamed": g(streamed, warm_ms),
           "warm_frac_streamed": f(streamed, warm_ms), "warm_GBps_sector": g(sector, warm_ms),
           "warm_frac_sector": f(sector, warm_ms),
           "cold_ms": round(cold_ms, 5), "cold_kernel_ms": round(cold_kernel_ms, 5) if cold_kernel_ms > 0 else None,
           "cold_frac_sector": f(sector, cold_ms),
           "traffic": traffic.get("bytes_per_launch") if traffic else None,
           "traffic_ratio_vs_sector": round(traffic["bytes_per_launch"] / sector, 3) if traffic else None,
           "traffic_source": traffic.get("source") if traffic else None}
    # test.py:12-17's solve on this family: GMRES(30) + Jacobi, a fixed 60
    # iterations (two restart cycles, rtol 0), through the column-block MatMult
    # and through the one-pass SELL kernel (key 84 = 0, reassembled)
    from mxsolve import _lib
    from mxsolve.core import rhs_hash
    b = comm.empty(m)
    rhs_hash(comm, 0, b)

    def gmres_rate(M):
        x = comm.zeros(m)
        M.solve(b, x, ksp="gmres", pc="jacobi", rtol=0.0, max_it=30)   # KSPSetUp, graph capture
        x.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = M.solve(b, x, ksp="gmres", pc="jacobi", rtol=0.0, max_it=60)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return {"its": r["its"], "its_per_s": round(r["its"] / dt, 1), "ms_per_it": round(dt * 1e3 / r["its"], 4)}

    out["gmres30_jacobi"] = {"column_block": gmres_rate(A)}
    A.destroy()
    L = _lib.load()
    old = L.mx_debug_set(84, 0)
    try:
        B = DMat.from_csr(comm, N, N, ip, cj, vv)
    finally:
        L.mx_debug_set(84, old)
    out["gmres30_jacobi"]["one_pass"] = gmres_rate(B)
    B.destroy()
    del ip, cj, vv, xt, y, b
    torch.cuda.empty_cache()
    return out


# The other BASELINE.json configurations on one GPU (C2, C4, C5's per-GPU
# share), reported beside the headline outside its timed region.  The
# expected iteration counts and reasons are the ones the full-size oracle
# parity tests pin (tests/test_gpu_fullsize.py: C2 7,723, C4 530, C5 share 245;
# all CONVERGED_RTOL) -- the driver run does not re-run the host oracle for them.
BENCH_CONFIGS = [("C2", "poisson2d", (4096, 4096, 1), "cg", (7723, 2)),
                 ("C4", "convdiff3d", (256, 256, 256), "gmres", (530, 2)),
                 ("C5share", "poisson3d27", (512, 512, 64), "cg", (245, 2))]


def kernel_frac(name: str, ms: float, count: int, nbytes: int) -> dict | None:
    """One kernel's roofline record: the mean of its dispatch-attached event
    times over `count` launches against its algorithmic bytes per launch."""
    if not count:
        return None
    avg = ms / count
    return {"kernel": name, "launches": count, "avg_launch_ms": round(avg, 5), "bytes_per_launch": int(nbytes),
            "GBps": round(nbytes / (avg * 1e-3) / 1e9, 1), "frac": round(nbytes / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def config_leg(comm, tag: str, kind: str, dims, ksp: str, expect) -> dict:
    """One BASELINE configuration on one GPU: device assembly (the stencil
    generator through the createAIJ pipeline) timed by phase with each phase's
    bytes, the converged solve (its and reason checked against the full-size
    parity tests' counts), time to solution, and the per-kernel HBM fractions
    from a profiled solve whose launches carry dispatch-attached HIP events
    (C2 / C5: CG mode 5's passes; C4: GMRES's MatMult, MDot and MAXPY)."""
    import torch
    from mxsolve.core import DMat, assembly_times, rhs_hash
    nx, ny, nz = dims
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    A = DMat.stencil(comm, kind, nx, ny, nz)
    torch.cuda.synchronize()
    t_asm = time.perf_counter() - t0
    ph = assembly_times()
    info = A.info()
    m, nnz = info["m"], info["nnz_d"] + info["nnz_o"]
    S = {"poisson2d": 5, "poisson3d27": 27}.get(kind, 7)
    gbs = lambda b, ms: round(b / (ms * 1e-3) / 1e9, 1) if ms > 0 else None
    # byte models of the phases (one rank): the generator writes S column
    # (cb = 4 bytes below 2^31 global rows, else 8) + fp64 slots per row and
    # the row pointer; the fused count pass reads the row pointer and the
    # columns and writes the A_d / A_o counts; the fused fill pass (split)
    # reads the row pointer, the slots and the split row pointers and writes
    # int32 columns + values and the diagonal; the layouts read A_d and write
    # the SELL values, read them back for the value codes and the row-pair codes
    cb = 4 if nx * ny * (1 if kind == "poisson2d" else nz) < 2 ** 31 else 8
    gen_canon_b = (2 * cb + 8) * S * m + 32 * m
    split_b = (cb + 8) * S * m + 12 * nnz + 32 * m
    layout_b = 12 * nnz + 8 * m + 3 * 8 * info["sell_slots_d"] + 2 * info["sell_slots_d"]
    asm = {"assembly_s": round(t_asm, 4),
           "phases": {"generate+canonicalise": {"ms": round(ph["canon_ms"], 3), "bytes": gen_canon_b,
                                                "GBps": gbs(gen_canon_b, ph["canon_ms"])},
                      "split": {"ms": round(ph["split_ms"], 3), "bytes": split_b, "GBps": gbs(split_b, ph["split_ms"])},
                      "layouts": {"ms": round(ph["layout_ms"], 3), "bytes_lower_bound": layout_b,
                                  "GBps": gbs(layout_b, ph["layout_ms"])}}}
    b = comm.empty(m)
    rhs_hash(comm, 0, b)
    x = comm.zeros(m)
    A.solve(b, x, ksp=ksp, pc="jacobi", rtol=0.0, max_it=20)       # KSPSetUp, PCSetUp, graph capture
    x.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = A.solve(b, x, ksp=ksp, pc="jacobi")
    torch.cuda.synchronize()
    ts = time.perf_counter() - t0
    kern = {}
    if ksp == "gmres":
        K = 60                                                          # two whole restart cycles
        x.zero_()
        rp = A.solve(b, x, ksp="gmres", pc="jacobi", rtol=0.0, max_it=K, profile=7)
        steps = [j % 30 for j in range(K)]
        mv = 16 * m + 4 * (m // 128)               # coded z-march, Jacobi by code: x in, w out, block ids
        kern["matmult"] = kernel_frac("spmv_pair_zmc_kernel<SPMV_JACOBI_S> (coded z-march MatMult + Jacobi)",
                                      rp["spmv_ms"], rp["spmv_count"], mv)
        mdot_b = sum(8 * m * (j + 2) for j in steps) / K
        maxpy_b = sum(8 * m * (j + 3) for j in steps) / K
        kern["mdot"] = kernel_frac("mdot_chunk_kernel (k+1 dots, one pass over w; mean over j = 0..29)",
                                   rp["mdot_ms"], rp["mdot_count"], mdot_b)
        kern["maxpy_norm"] = kernel_frac("maxpy_norm_kernel (VecMAXPY + ||w||^2; mean over j = 0..29)",
                                         rp["maxpy_ms"], rp["maxpy_count"], maxpy_b)
    else:
        x.zero_()
        rp = A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=100, profile=15)
        xb = rp.get("cg_xbatch", 1)
        meta = pair_meta_bytes(info, m, nnz, info["nghost"])
        if rp["cg_mode"] == 5:
            kern["residual_update"] = kernel_frac("CG mode 5 residual update (A p recomputed, r read and written)",
                                                  rp["upd_ms"], rp["upd_count"], 24 * m + meta)
            kern["pAp_pass"] = kernel_frac("CG mode 5 p.Ap pass (p read, nothing stored)",
                                           rp["spmv_ms"], rp["spmv_count"], 8 * m + meta)
            kern["direction_pAp_fused"] = kernel_frac("spmv_pair_pbw_kernel (p_i = z + b p_(i-1) formed and "
                                                      "stored, p.Ap partials)", rp["pbw_ms"], rp["pbw_count"],
                                                      24 * m + meta)
        pb_bytes = ((24 + 8 * (xb - 1) + 16) * m if rp.get("pbw_count") else
                    24 * m + (8 * (xb - 1) + 16) * m // max(xb, 1))
        kern["direction_update"] = kernel_frac(f"cg_pb_kernel (direction update, x steps batched by {xb}"
                                               + ("; batch launches only" if rp.get("pbw_count") else "") + ")",
                                               rp["pb_ms"], rp["pb_count"], pb_bytes)
    A.destroy()
    del b, x
    torch.cuda.empty_cache()
    return {"config": tag, "workload": f"{kind} {nx}x{ny}x{nz}, {ksp.upper()}" + ("(30)" if ksp == "gmres" else "")
            + " + Jacobi, fp64, one GPU", "rows": m, "nnz": nnz,
            "its": r["its"], "reason": r["reason"], "expected_its_reason": list(expect),
            "parity_counts_ok": (r["its"], r["reason"]) == tuple(expect),
            "solve_s": round(ts, 4), "its_per_s": round(r["its"] / ts, 1),
            "time_to_solution_s": round(t_asm + ts, 4), **asm,
            "cg_mode": r.get("cg_mode") if ksp == "cg" else None,
            "kernels": {k: v for k, v in kern.items() if v}}


def oracle_check(grid: int, P: int, threads: int) -> dict:
    """The parity checker (not measured): the oracle's C restatement of PETSc's
    CG + Jacobi (oracle/petsc_oracle.c, P-rank row-block model) solving the
    same grid^3 system to convergence; returns its x, its and reason."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    ip, c, v = oracle.stencil("poisson3d", grid)
    M = ip.size - 1
    A = oracle.OracleMat.from_csr(M, M, ip, c, v, P=P)
    del ip, c, v
    b = oracle.rhs_hash(0, M)
    t0 = time.perf_counter()
    r = A.solve(b, ksp="cg", pc="jacobi", nthreads=threads)
    return {"x": r["x"], "its": int(r["its"]), "reason": int(r["reason"]), "P": P,
            "solve_s": round(time.perf_counter() - t0, 3)}


PARITY_BAR = "its and reason equal to the oracle's, x within relative L2 1e-10 (north_star)"


def choose_leg(legs: list, no_solve: bool = False) -> dict:
    """The leg `value` is taken from: the fastest whose converged solve
    passed the parity check (every leg when no converged solves ran); when
    none passed, the first leg -- its parity record then says so."""
    passing = [lg for lg in legs if lg.get("parity", {}).get("ok", no_solve)]
    return max(passing or legs[:1], key=lambda lg: lg["value"])


def rnd(v, k):
    return None if v is None else round(v, k)


# Wall-time budget of one timed leg (seconds; MXSOLVE_BENCH_LEG_BUDGET_S).  A
# leg normally takes a few seconds (RCCL warm-up, W + K iterations, the
# converged solve); a hung one (a multi-rank RCCL graph capture that never
# completes, a peer that never arrives) must not eat the driver's run.
LEG_BUDGET_S = 60.0


class LegWatchdog:
    """Backstop of one leg's budget: a timer that calls `abort` (mx_comm_abort:
    ncclCommAbort / the shared-memory world's abort flag) when the leg is still
    running `after_s` seconds in, for a rank blocked somewhere that does not
    poll a deadline of its own (the library's waits already fail after knobs
    33 / 47, which run_legs sets to the budget).  The blocked call then fails
    with MX_ERR_COMM and the leg is recorded as failed."""

    def __init__(self, after_s: float, abort):
        import threading
        self.fired = False
        self._abort = abort
        self._t = threading.Timer(after_s, self._fire)
        self._t.daemon = True

    def _fire(self):
        self.fired = True
        try:
            self._abort()
        except Exception:  # noqa: BLE001  (the blocked call reports the failure)
            pass

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._t.cancel()
        return False


def run_legs(specs, run_leg, set_knobs, budget_s: float, abort, err_type):
    """Run the timed legs in order under a wall-time budget each.  Per leg the
    library's deadlines -- knob 33 (no progress in a solve) and knob 47 (plain
    stream waits) -- are set to the budget unless the leg sets its own, and a
    LegWatchdog aborts the communicator at twice the budget.  A leg that fails
    (MX_ERR_COMM: an RCCL error, a deadline, the watchdog) ends the loop: the
    communicator is aborted, so no later leg or collective can run; the line is
    then printed from the legs already measured (the first leg failing raises:
    there is nothing to report).  Returns (legs, failed, comm_dead)."""
    legs, failed, dead = [], [], None
    dl = int(budget_s * 1000)
    for name, kn in specs:
        old = set_knobs({33: dl, 47: dl, **kn})
        t0 = time.perf_counter()
        wd = LegWatchdog(2 * budget_s, abort)
        try:
            with wd:
                leg = run_leg(name, kn)
            leg["wall_s"] = round(time.perf_counter() - t0, 3)
            legs.append(leg)
        except err_type as e:
            if not legs:
                raise
            failed.append({"leg": name, "knobs": kn, "error": str(e), "wall_s": round(time.perf_counter() - t0, 3),
                           "budget_s": budget_s, "watchdog_fired": wd.fired})
            dead = str(e)
            break
        finally:
            set_knobs(old)
    return legs, failed, dead


def parse_stall(spec: str | None):
    """MXSOLVE_BENCH_STALL_LEG=<leg name>:<seconds> -- rehearsal hook: in that
    leg the last rank sleeps before the timed solve (a peer that stops
    answering), so the budget can be exercised."""
    if not spec or ":" not in spec:
        return None
    name, s = spec.rsplit(":", 1)
    return name, float(s)


def parity_record(its: int, reason: int, rel: float, o: dict) -> dict:
    return {"checker": f"oracle/petsc_oracle.c CG + Jacobi, P = {o['P']} row-block model, converged "
                       f"(rtol 1e-5), {o['solve_s']} s on the host",
            "gpu_its": int(its), "oracle_its": o["its"], "gpu_reason": int(reason), "oracle_reason": o["reason"],
            "its_equal": int(its) == o["its"], "reason_equal": int(reason) == o["reason"],
            "rel_l2": float(f"{rel:.3e}"), "bar": PARITY_BAR,
            "ok": int(its) == o["its"] and int(reason) == o["reason"] and rel <= 1e-10}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-solve", action="store_true", help="skip the converged solves and the parity check")
    ap.add_argument("--no-asm", action="store_true", help="skip the createAIJ-from-host-arrays leg")
    ap.add_argument("--no-general", action="store_true", help="skip the streamed-values SpMV leg (spmv_general)")
    ap.add_argument("--no-configs", action="store_true", help="skip the C2 / C4 / C5-share configuration legs")
    ap.add_argument("--no-random", action="store_true", help="skip the random-pattern (unstructured AIJ) SpMV leg")
    ap.add_argument("--cpu-config", choices=sorted(CPU_CONFIGS),
                    help="only the host (oracle) baseline of another BASELINE configuration: one JSON line")
    args = ap.parse_args()
    if args.cpu_config:
        threads, how = cpu_threads()
        print(json.dumps(cpu_baseline_config(args.cpu_config, threads, how)), flush=True)
        return

    import numpy as np
    import torch
    from mxsolve import _lib
    from mxsolve.core import DeviceComm, DMat, rhs_hash, unique_id
    L = _lib.load()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    shm = os.environ.get("MXSOLVE_TRANSPORT", "").lower() == "shm"
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        if shm:
            # rehearsal of the N > 1 flow with ranks sharing a GPU (host-staged
            # transport, not a measurement): the driver's runs use RCCL
            import secrets
            name = [f"/mxsolve_bench_{secrets.token_hex(6)}" if rank == 0 else None]
            dist.broadcast_object_list(name, src=0)
            comm = DeviceComm.shm(rank, world, name[0], device=local % torch.cuda.device_count())
        else:
            uid = [unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = DeviceComm.rccl(rank, world, uid[0], device=local)
    else:
        comm = DeviceComm.self_comm(local)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    def max_over_ranks(v: float) -> float:
        if dist is None:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    def sum_over_ranks(vals):
        t = torch.tensor(vals, dtype=torch.float64)
        if dist is not None:
            dist.all_reduce(t)
        return t.tolist()

    def gather(obj):
        if dist is None:
            return [obj]
        got = [None] * world
        dist.all_gather_object(got, obj)
        return got

    n = args.grid
    # process start-up, not assembly: the first launches of the library load
    # its code objects and the allocator maps its first pools -- paid once per
    # process (PetscInitialize's share), so a small operator takes it here
    barrier()
    t0 = time.perf_counter()
    A0 = DMat.stencil(comm, "poisson3d", 8)
    b0 = comm.empty(A0.info()["m"])
    rhs_hash(comm, A0.info()["rstart"], b0)
    x0 = comm.zeros(A0.info()["m"])
    A0.solve(b0, x0, ksp="cg", pc="jacobi", rtol=0.0, max_it=2)
    A0.destroy()
    del b0, x0
    barrier()
    t_init = max_over_ranks(time.perf_counter() - t0)
    barrier()
    t0 = time.perf_counter()
    A = DMat.stencil(comm, "poisson3d", n)
    barrier()
    t_asm = max_over_ranks(time.perf_counter() - t0)
    info = A.info()
    m, nnz_loc, ng = info["m"], info["nnz_d"] + info["nnz_o"], info["nghost"]
    b = comm.empty(m)
    rhs_hash(comm, info["rstart"], b)
    x = comm.zeros(m)

    # first solve on the fresh operator pays PCSetUp_Jacobi (diagonal, the
    # uniform-diagonal test) and KSPSetUp (work space): time it against a repeat
    barrier()
    t0 = time.perf_counter()
    A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=1)
    barrier()
    t_first = time.perf_counter() - t0
    t0 = time.perf_counter()
    A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=1)
    barrier()
    t_setup = max_over_ranks(max(t_first - (time.perf_counter() - t0), 0.0))

    # The timed legs.  One rank: the library's own choice (CG mode 5, graph
    # replay).  N > 1: the open choices are measured here rather than taken
    # from the one-GPU proxy -- the fusion mode (knob 9: 2 = stored product,
    # 5 = recomputed product) times eager launches or RCCL graph replay (knob 7
    # = 1 / 2); value comes from the fastest leg whose converged solve passes
    # the parity check.  Each leg: W untimed iterations, then exactly K timed
    # between barrier + sync on both sides (rtol = 0 never stops early), max
    # over ranks; then the leg's converged solve (default tolerances) whose
    # its, reason and x are checked against the oracle below.
    if world == 1:
        leg_specs = [("auto", {})]
    else:
        # the library's default first ("auto": CG mode 5 with the direction
        # update fused into the split p.Ap pass where it applies, else mode 2;
        # eager launches), then the alternatives: mode 2, mode 5 with the
        # separate direction update pass (knob 80 = 0, the same bits), and
        # last the RCCL graph-replay legs -- a multi-rank RCCL capture has
        # only ever run on the driver's node, so if it fails or hangs there,
        # the eager legs are already measured and the line is still printed
        # from them (every leg runs under a wall-time budget: run_legs)
        leg_specs = [("auto", {}), ("mode2/eager", {9: 2, 7: 1}),
                     ("mode5sep/eager", {9: 5, 80: 0, 7: 1}),
                     ("mode2/graph", {9: 2, 7: 2, 33: 30000}), ("mode5/graph", {9: 5, 7: 2, 33: 30000})]

    def set_knobs(kn):
        return {k: L.mx_debug_set(k, v) for k, v in kn.items()}

    stall = parse_stall(os.environ.get("MXSOLVE_BENCH_STALL_LEG"))

    def run_leg(name, kn):
        # rehearsal hook: the failure path of a leg (MXSOLVE_BENCH_FAIL_LEG=<leg name>)
        if os.environ.get("MXSOLVE_BENCH_FAIL_LEG") == name:
            raise _lib.MxError(_lib.MX_ERR_COMM, f"injected failure of leg {name}")
        if args.warmup > 0:
            A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=args.warmup)
        barrier()
        if stall and stall[0] == name and rank == world - 1:
            time.sleep(stall[1])             # rehearsal hook: a peer that stops answering
        t0 = time.perf_counter()
        r = A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=args.steps)
        barrier()
        dt_local = time.perf_counter() - t0
        dt = max_over_ranks(dt_local)
        assert r["its"] == args.steps, r
        leg = {"leg": name, "knobs": kn, "cg_mode": r["cg_mode"], "cg_xbatch": r["cg_xbatch"],
               "value": round(args.steps / dt, 3),
               "ms_per_step": round(dt / args.steps * 1e3, 4), "_dt": dt,
               "per_rank_timed_s": [round(v, 5) for v in gather(dt_local)]}
        if not args.no_solve:
            x.zero_()
            barrier()
            t0 = time.perf_counter()
            rs = A.solve(b, x, ksp="cg", pc="jacobi")
            barrier()
            ts = max_over_ranks(time.perf_counter() - t0)
            leg.update({"its": rs["its"], "reason": rs["reason"], "solve_s": ts, "_x": x.clone()})
        return leg

    budget = float(os.environ.get("MXSOLVE_BENCH_LEG_BUDGET_S", LEG_BUDGET_S))
    legs, failed, comm_dead = run_legs(leg_specs, run_leg, set_knobs, budget,
                                       lambda: L.mx_comm_abort(comm.h) if world > 1 else None, _lib.MxError)

    # parity: every leg's converged solve against the oracle (the checker, run
    # on rank 0 after the GPU work; at N = 1 it is the cpu_baseline leg's own
    # converged oracle solve).  N > 1: rank 0 broadcasts the oracle's x and
    # every rank compares its own rows.
    cpu = None
    threads, how = cpu_threads()
    if not args.no_solve:
        o = None
        if rank == 0:
            if world == 1 and not args.no_cpu:
                cpu = cpu_baseline(n, threads, how)
                o = cpu.pop("_oracle")
            else:
                o = oracle_check(n, world, threads)
        ox = o["x"] if rank == 0 else None
        if dist is not None:
            meta = [None if rank else {k: v for k, v in o.items() if k != "x"}]
            dist.broadcast_object_list(meta, src=0)
            t = torch.from_numpy(ox) if rank == 0 else torch.empty(info["M"], dtype=torch.float64)
            dist.broadcast(t, src=0)
            o, ox = dict(meta[0]), t.numpy()
        xo = torch.from_numpy(np.ascontiguousarray(ox[info["rstart"]:info["rstart"] + m])).to(x.device)
        for leg in legs:
            d = leg.pop("_x")
            s2 = sum_over_ranks([float(torch.sum((d - xo) ** 2)), float(torch.sum(xo * xo))])
            rel = (s2[0] ** 0.5) / max(s2[1] ** 0.5, 1e-300)
            leg["parity"] = parity_record(leg["its"], leg["reason"], rel, o)
            del d
        del xo, ox
    elif rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(n, threads, how)
        cpu.pop("_oracle")
    chosen = choose_leg(legs, args.no_solve)
    set_knobs(chosen["knobs"])          # the chosen leg's settings for the measurements below
    value, dt = chosen["value"], chosen["_dt"]
    legs += failed

    mode, xb = chosen["cg_mode"], chosen.get("cg_xbatch", 1)
    bytes_csr = spmv_bytes(m, nnz_loc, ng)
    bytes_spmv = spmv_format_bytes(info, m, nnz_loc, ng)
    pw = dom = comm_lat = None
    achieved = avg_ms = spmv_avg_ms = spmv_alone_ms = mult_ms = cold_ms = cold_kernel_ms = bytes_launch = None
    if comm_dead is None:       # (an aborted communicator runs nothing more)
        # roofline pass: the same CG iterations with a HIP event pair on every
        # MatMult-family launch (on the library stream the kernel runs on; one
        # rank: the events are attached to the kernel's own dispatch by
        # hipExtLaunchKernel, so they time the kernel alone, as the profiler's
        # trace does).  Kept out of the K timed steps: the profiled solve runs
        # eagerly (no graph).  profile bit 0: the MatMult (mode 5: the p.Ap pass),
        # bit 1: mode 5's residual update, bit 2: the batched direction update
        x.zero_()
        rp = A.solve(b, x, ksp="cg", pc="jacobi", rtol=0.0, max_it=min(args.steps, 100), profile=15)
        mode = rp["cg_mode"]
        xb = rp.get("cg_xbatch", 1)
        spmv_avg_ms = rp["spmv_ms"] / max(rp["spmv_count"], 1)
        bytes_csr = spmv_bytes(m, nnz_loc, ng)
        bytes_spmv = spmv_format_bytes(info, m, nnz_loc, ng)
        meta = pair_meta_bytes(info, m, nnz_loc, ng)
        pw = None
        if mode == 5:
            # the SpMV-bearing kernel: the residual update (A p recomputed, r read
            # and written); the p.Ap pass reported beside it
            upd_avg_ms = rp["upd_ms"] / max(rp["upd_count"], 1)
            bytes_launch = 8 * (m + ng) + 16 * m + meta
            avg_ms = upd_avg_ms
            bytes_pw = 8 * (m + ng) + meta
            pw = {"kernel": "spmv_pair_zm_kernel<SPMV_PW> (p.Ap partials, product not stored)",
                  "avg_launch_ms": round(spmv_avg_ms, 5), "bytes_per_launch": bytes_pw,
                  "GBps": round(bytes_pw / (spmv_avg_ms * 1e-3) / 1e9, 1),
                  "frac": round(bytes_pw / (spmv_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                  # the direction update fused into the p.Ap pass (knob 69; off at 256^3):
                  # r and p_(i-1) in, p_i out
                  "fused_direction_pass": kernel_frac("spmv_pair_pbw_kernel" if world == 1 else
                                                      "cg5_pbws_matmult (halo pack + fused split p.Ap pass + "
                                                      "boundary kernel, HIP events around them)",
                                                      rp["pbw_ms"], rp["pbw_count"], 24 * m + meta)}
        else:
            bytes_launch = bytes_spmv + (32 * m if mode == 1 else 0)   # SPMV_CG: + r, x r/w, p_i
            avg_ms = spmv_avg_ms
        achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
        # the direction update (the iteration's longest kernel in mode 5): r and
        # p_{i-1} in, p_i out (24 B/row), and every xb-th launch the xb - 1 older
        # directions and x in, x out -- per launch on average 24 + (8 (xb - 1) + 16) / xb B/row
        dom = None
        if rp.get("pb_count"):
            pb_ms = rp["pb_ms"] / rp["pb_count"]
            # with the fused direction + p.Ap pass (knob 69) the direction
            # update runs only on the x-batch iterations: every launch a batch one
            pb_bytes = ((24 + 8 * (xb - 1) + 16) * m if rp.get("pbw_count") else
                        24 * m + (8 * (xb - 1) + 16) * m // max(xb, 1))
            dom = {"kernel": f"cg_pb_kernel<JM, {xb}> (direction update p_i = z + b p_(i-1), the x steps batched by {xb})",
                   "avg_launch_ms": round(pb_ms, 5), "launches": rp["pb_count"], "bytes_per_launch": pb_bytes,
                   "GBps": round(pb_bytes / (pb_ms * 1e-3) / 1e9, 1),
                   "frac": round(pb_bytes / (pb_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
            tp = load_traffic(n, world, mode, "/pb")
            dom.update({"traffic": tp["bytes_per_launch"] if tp else None,
                        "traffic_source": tp.get("source") if tp else None})
        # standalone SpMV timing (same kernel, back-to-back)
        y = comm.empty(m)
        spmv_alone_ms, mult_ms = A.bench_mult(b, y, 50)
        # cold-cache MatMult: 1 GB streamed through the caches first (SURVEY
        # §8d), the MatMult queued behind it by the library (no host launch
        # gap inside the span; round 5's torch events around A.mult() held one)
        flush = torch.empty(1 << 27, dtype=torch.float64, device=y.device)
        cold_kernel_ms, cold_ms = A.bench_mult_cold(b, y, flush, 5)
        del flush

        # communication latency on the library stream (N > 1): the two CG
        # all-reduces and the halo exchange, back to back; diagnostics for scaling
        comm_lat = None
        if world > 1:
            comm_lat = {"allreduce_1_us": round(comm.comm_bench(0, 200), 2),
                        "allreduce_3_us": round(comm.comm_bench(1, 200), 2),
                        "halo_us": round(comm.comm_bench(2, 200, A), 2)}

    solve = None
    if "its" in chosen:
        ts = chosen["solve_s"]
        solve = {"its": chosen["its"], "reason": chosen["reason"], "time_s": round(ts, 4),
                 "its_per_s": round(chosen["its"] / ts, 2), "assembly_s": round(t_asm, 3),
                 "pcsetup_kspsetup_s": round(t_setup, 4),
                 "time_to_solution_s": round(ts + t_asm + t_setup, 3),
                 "process_init_s": round(t_init, 3)}

    copy_gbps = round(stream_copy_gbps(x.device, m), 1) if comm_dead is None else None

    asm_host = None
    if rank == 0 and world == 1 and not args.no_asm:
        asm_host = assembly_from_host(comm, n, n, n)

    general = None
    if rank == 0 and world == 1 and not args.no_general:
        general = spmv_general_leg(comm, n)

    random_leg = None
    if rank == 0 and world == 1 and not args.no_random:
        random_leg = spmv_random_leg(comm)

    configs = None
    if rank == 0 and world == 1 and not args.no_configs:
        configs = [config_leg(comm, *c) for c in BENCH_CONFIGS]

    iter_bytes = cg_iter_bytes_design(info, m, nnz_loc, ng, mode, xb)
    # the library's default residual update at this size (mx_spmv_pair.hip
    # pair_cg5_rupd_launch, knob 68 = 3: two lines per wave from 2^23 rows)
    two_line = world == 1 and mode == 5 and m >= (1 << 23) and info.get("pair_shape") == 7
    iter_gbps = iter_bytes * value / 1e9
    if rank == 0:
        traffic = load_traffic(n, world, mode)
        for lg in legs:
            lg.pop("_dt", None)
            if "solve_s" in lg:
                lg["solve_s"] = round(lg["solve_s"], 4)
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "CG iterations/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"3D 7-point Poisson {n}^3, CG + Jacobi, fp64, row-block partitioned",
                       "rows": info["M"], "nnz": int(7 * n**3 - 6 * n**2),
                       "parallelism": (f"row-block x{world} (" + ("shared-memory rehearsal" if shm else "RCCL halo + allreduce") + ")") if world > 1 else "single GPU"},
            "parity": chosen.get("parity"),
            "roofline": {"bound": "hbm", "achieved": rnd(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": rnd(achieved and achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic["bytes_per_launch"] if traffic else None,
                         "traffic_source": (traffic.get("source", "") + " -- rocprofv3 PMC (FETCH_SIZE x 2 + "
                                            "WRITE_SIZE, gfx950 correction) of the same kernel on a builder box, "
                                            "not counters of this run") if traffic else None,
                         "traffic_detail": traffic,
                         "kernel": (("spmv_pair_zm2l_kernel<JM, 5> (two lines per wave, knob 68; " if two_line else
                                     "spmv_pair_zm_kernel<SPMV_RUPD> (") +
                                    "CG mode 5 residual update only: r -= alpha A p "
                                    "with A p recomputed, [z.z, z.r, r.r] folded" if mode == 5 else
                                    "spmv_sell_kernel<SPMV_CG> (CG-fused MatMult" if mode == 1 else
                                    ("spmv_pair_zm_kernel<SPMV_DOT> (CG MatMult, lean row-pair z-march" if info.get("pair_zmarch") else
                                     "spmv_pair_lean_kernel<SPMV_DOT> (CG MatMult, lean row-pair" if info.get("pair_lean") else
                                     "spmv_sell_kernel<SPMV_DOT> (CG MatMult")) +
                                   (", HIP events attached to the kernel's dispatch (hipExtLaunchKernel)" if world == 1 else
                                    ", HIP events around the MatMult") + ", rank 0)",
                         "bytes_per_launch": bytes_launch, "avg_launch_ms": rnd(avg_ms, 5),
                         "format": ("value codes (" + str(info.get("value_codes")) + " distinct), " +
                                    ("row pairs" if info.get("pair_shape") else "one row per lane") +
                                    (f", {info['pair_blocks']} distinct code blocks" if info.get("pair_blocks") else "") +
                                    (" (uniform slots: values + lane masks)" if info.get("pair_uniform") else ""))
                                   if info.get("value_codes") else "fp64 SELL-64",
                         # the iteration's longest kernel, and the whole timed iteration
                         "dominant_kernel": dom,
                         "iteration": {"bytes": iter_bytes, "GBps": round(iter_gbps, 1),
                                       "frac": round(iter_gbps / HBM_PEAK_GBS, 4)},
                         # how much faster than a CSR SpMV (SURVEY §8d bytes) streaming at HBM peak
                         "csr_bytes_per_launch": bytes_csr,
                         "speedup_vs_csr_at_peak": rnd(spmv_avg_ms and (bytes_csr / (HBM_PEAK_GBS * 1e9)) / (spmv_avg_ms * 1e-3), 3)},
            "comm_failure": comm_dead,
            "pw_pass": pw,
            "cpu_baseline": cpu,
            "legs": legs,
            "converged_its_per_s": solve["its_per_s"] if solve else None,
            "stream_copy_GBps": copy_gbps,
            "spmv_standalone": {"avg_ms": round(spmv_alone_ms, 5),
                                "GBps": round(bytes_spmv / (spmv_alone_ms * 1e-3) / 1e9, 1),
                                "matmult_ms": round(mult_ms, 5),
                                "cold_matmult_ms": round(cold_ms, 5),
                                "cold_kernel_ms": round(cold_kernel_ms, 5) if cold_kernel_ms > 0 else None,
                                "cold_GBps": round(bytes_spmv / (cold_ms * 1e-3) / 1e9, 1),
                                "cold_frac": round(bytes_spmv / (cold_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                # the kernel alone (dispatch-attached events): the span above also
                                # holds the queue gap between the flush kernel's end and its start
                                "cold_kernel_frac": round(bytes_spmv / (cold_kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                if cold_kernel_ms and cold_kernel_ms > 0 else None}
            if spmv_alone_ms else None,
            "spmv_general": general,
            "spmv_random": random_leg,
            "cg_iter_bytes_survey": cg_iter_bytes(m, nnz_loc, ng),
            "cg_fusion_mode": mode,
            "cg_xbatch": xb,
            "cg_iter_bytes_alg": iter_bytes,
            "cg_iter_GBps_alg": round(iter_gbps, 1),
            # the whole timed iteration (every kernel, the per-solve start and
            # finish included) on its algorithmic bytes against HBM peak
            "cg_iter_frac": round(iter_gbps / HBM_PEAK_GBS, 4),
            "comm_latency": comm_lat,
            "solve": solve,
            "assembly_host_csr": asm_host,
            "configs": configs,
        }
        print(json.dumps(out), flush=True)
    try:
        A.destroy()
        comm.destroy()
    except _lib.MxError:
        if comm_dead is None:
            raise
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
