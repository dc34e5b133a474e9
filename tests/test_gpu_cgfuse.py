"""CG with the direction update and the x step fused into the MatMult
(SPMV_CG, knob 9) against the separate-pass iteration: identical bits in x,
the residual history, the iteration count and the reason -- on one rank, on
2 and 4 in-process ranks with the overlapped halo, for uniform and variable
Jacobi, no preconditioner, every norm type, a nonzero guess, max_it limits
and an indefinite stop.  Both are checked against the oracle elsewhere."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _single_row_layout():
    """These tests compare CG variants bit for bit; the row-pair MatMult
    (knob 27) sums the dot partials per lane over a different row grouping,
    so it is held at the single-row layout here (it is checked against the
    oracle in test_gpu_vcodes.py)."""
    from mxsolve import _lib
    old = _lib.load().mx_debug_set(27, 0)
    yield
    _lib.load().mx_debug_set(27, old)


def _knob(v):
    from mxsolve import _lib
    return _lib.load().mx_debug_set(9, v)


def _mat(comm, oracle, kind):
    from mxsolve.core import DMat
    if kind == "varidiag":         # SPD, non-uniform diagonal: the vector Jacobi path
        ip, c, v = oracle.stencil("poisson3d", 12)
        M = ip.size - 1
        rows = np.repeat(np.arange(M), np.diff(ip))
        d = 1.0 + np.random.default_rng(3).random(M)
        R = np.concatenate([rows, np.arange(M)])
        Cc = np.concatenate([c, np.arange(M)])
        V = np.concatenate([v, d])
        r0, r1 = oracle.split_ownership(M, comm.size)[comm.rank:comm.rank + 2]
        sel = (R >= r0) & (R < r1)
        return DMat.from_coo(comm, M, M, R[sel], Cc[sel], V[sel], add=True)
    if kind == "indef":
        M = 40
        d = np.linspace(4.0, -1.0, M)
        r0, r1 = oracle.split_ownership(M, comm.size)[comm.rank:comm.rank + 2]
        idx = np.arange(r0, r1)
        return DMat.from_coo(comm, M, M, idx, idx, d[r0:r1])
    if kind == "odd":              # 13^3 = 2197 rows: the paired walk's tail row
        return DMat.stencil(comm, "poisson3d", 13)
    return DMat.stencil(comm, kind, 14)


def _run(comm, oracle, kind, fuse, **kw):
    old = _knob(fuse)
    try:
        return _solve(comm, oracle, kind, **kw)
    finally:
        _knob(old)


def _solve(comm, oracle, kind, **kw):
    from mxsolve.core import rhs_hash
    if True:
        A = _mat(comm, oracle, kind)
        info = A.info()
        b = comm.empty(info["m"])
        rhs_hash(comm, info["rstart"], b)
        x = comm.zeros(info["m"])
        if kw.pop("negzero", False):     # -0.0 entries: p_0 = z keeps the sign of zero
            b[::5] = -0.0
        if kw.pop("guess", False):
            rhs_hash(comm, info["rstart"] + 7, x)
            x.mul_(0.25)
            kw["guess_nonzero"] = True
        r = A.solve(b, x, ksp="cg", history=True, **kw)
        A.destroy()
        return r["its"], r["reason"], r["history"], x.cpu().numpy()


CASES = [("poisson3d", {}), ("poisson3d", {"max_it": 7}), ("poisson3d", {"max_it": 16}),
         ("poisson3d", {"pc": "none"}), ("poisson3d", {"norm": "unpreconditioned"}),
         ("poisson3d", {"norm": "natural"}), ("poisson3d", {"norm": "none", "max_it": 20}),
         ("poisson3d", {"guess": True}), ("poisson3d27", {}), ("varidiag", {}),
         ("varidiag", {"max_it": 5}), ("indef", {"pc": "none"}), ("poisson3d", {"negzero": True, "max_it": 3})]


def _same(a, b):
    assert (a[0], a[1]) == (b[0], b[1])
    assert np.array_equal(a[2].view(np.uint64), b[2].view(np.uint64))
    assert np.array_equal(a[3].view(np.uint64), b[3].view(np.uint64))


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("kind,kw", CASES)
def test_fused_equals_separate_one_rank(selfcomm, oracle_mod, kind, kw, mode):
    _same(_run(selfcomm, oracle_mod, kind, mode, **dict(kw)), _run(selfcomm, oracle_mod, kind, 0, **dict(kw)))


@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("kind,kw", [("poisson3d", {}), ("varidiag", {}), ("poisson3d", {"max_it": 9})])
def test_fused_equals_separate_ranks(oracle_mod, P, kind, kw):
    from mxsolve.core import LocalWorld
    outs = {}
    for fuse in (1, 2, 0):
        w = LocalWorld(P)
        old = _knob(fuse)          # set once, outside the rank threads
        try:
            outs[fuse] = w.run(lambda comm: _solve(comm, oracle_mod, kind, **dict(kw)))
        finally:
            _knob(old)
            w.destroy()
    for mode in (1, 2):
        for a, b in zip(outs[mode], outs[0]):
            _same(a, b)


@pytest.mark.parametrize("P", [3])
def test_fused_equals_separate_three_ranks(oracle_mod, P):
    """P = 3 with the overlapped halo (the boundary launch folds the partials
    of both MatMult launches in-launch): CG mode 1 gives mode 0's bits.
    (Round 5's fold placements 0/2/3, knob 10, are retired: the update pass
    folds in-launch, the split MatMult's boundary launch too.)"""
    from mxsolve.core import LocalWorld
    outs = {}
    for fuse in (0, 1):
        w = LocalWorld(P)
        o9 = _knob(fuse)
        try:
            outs[fuse] = w.run(lambda comm: _solve(comm, oracle_mod, "poisson3d", **{}))
        finally:
            _knob(o9)
            w.destroy()
    for a, b in zip(outs[1], outs[0]):
        _same(a, b)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("kind,kw", [("poisson3d", {}), ("varidiag", {}), ("poisson3d", {"guess": True}),
                                     ("poisson3d", {"pc": "none", "max_it": 11}), ("odd", {}),
                                     ("odd", {"pc": "none"})])
def test_paired_vector_walk(selfcomm, oracle_mod, kind, kw, mode):
    """The row-pair walk of the CG vector passes (knob 13, 16-B accesses; odd
    row counts take a tail row) sums the partials in another order: same
    iterations and reason, x within 1e-12 of the row walk."""
    from mxsolve import _lib
    L = _lib.load()
    old = L.mx_debug_set(13, 1)
    try:
        a = _run(selfcomm, oracle_mod, kind, mode, **dict(kw))
    finally:
        L.mx_debug_set(13, old)
    b = _run(selfcomm, oracle_mod, kind, mode, **dict(kw))
    assert (a[0], a[1]) == (b[0], b[1])
    assert np.linalg.norm(a[3] - b[3]) <= 1e-12 * np.linalg.norm(b[3])


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("kind,kw", [("poisson3d", {}), ("varidiag", {}), ("odd", {"guess": True}),
                                     ("poisson3d", {"max_it": 9})])
def test_unrolled_row_walk_bitwise(selfcomm, oracle_mod, kind, kw, mode):
    """Four-step load batches in the CG vector passes (knob 21) keep each
    thread's sum order: bitwise the plain row walk."""
    from mxsolve import _lib
    L = _lib.load()
    out = {}
    for u in (0, 1):
        old = L.mx_debug_set(21, u)
        try:
            out[u] = _run(selfcomm, oracle_mod, kind, mode, **dict(kw))
        finally:
            L.mx_debug_set(21, old)
    _same(out[0], out[1])


@pytest.mark.parametrize("B", [2, 4])
@pytest.mark.parametrize("kind,kw", [("poisson3d", {}), ("poisson3d", {"max_it": 7}), ("poisson3d", {"max_it": 9}),
                                     ("poisson3d", {"max_it": 16}), ("varidiag", {}), ("poisson3d", {"guess": True}),
                                     ("indef", {"pc": "none"}), ("poisson3d27", {}), ("odd", {})])
def test_batched_x_steps_equal_separate(selfcomm, oracle_mod, kind, kw, B):
    """Mode 2 with the x steps applied every B iterations (knob 29): the same
    FMAs in the same order, so x and the history are identical to mode 0 for
    every stop position relative to the batch (max_it 7, 9, 16, convergence)."""
    from mxsolve import _lib
    L = _lib.load()
    old = L.mx_debug_set(29, B)
    try:
        a = _run(selfcomm, oracle_mod, kind, 2, **dict(kw))
    finally:
        L.mx_debug_set(29, old)
    _same(a, _run(selfcomm, oracle_mod, kind, 0, **dict(kw)))


@pytest.mark.parametrize("kind,n,pc,max_it,kw", [("poisson3d", 128, "jacobi", 10000, {}),
                                                 ("poisson3d", 64, "jacobi", 10000, {}),
                                                 ("poisson2d", 256, "none", 10000, {}),
                                                 ("poisson3d", 128, "jacobi", 37, {}),
                                                 ("poisson3d", 128, "jacobi", 1, {}),
                                                 ("poisson3d", 128, "jacobi", 2, {}),
                                                 ("poisson2d", 384, "jacobi", 10000, {}),
                                                 ("poisson3d", 128, "jacobi", 10000, {"guess": True}),
                                                 ("poisson3d", 128, "jacobi", 10000, {"norm": "natural"}),
                                                 ("poisson3d", 128, "jacobi", 10000, {"norm": "unpreconditioned"}),
                                                 ("poisson3d", 128, "jacobi", 10000, {"xb": 2}),
                                                 ("poisson3d", 128, "jacobi", 39, {"xb": 2}),
                                                 ("poisson3d", 128, "jacobi", 38, {}),
                                                 ("poisson3d27", 128, "jacobi", 10000, {}),
                                                 ("poisson3d27", 128, "jacobi", 37, {}),
                                                 ("poisson3d27", 128, "none", 10000, {"guess": True}),
                                                 ("poisson3d27", 128, "jacobi", 39, {"xb": 2}),
                                                 ("poisson3d27", 128, "jacobi", 10000, {"sym": 0}),
                                                 ("poisson3d27", 128, "jacobi", 10000, {"sym": 0, "k60": 0}),
                                                 ("poisson3d", 128, "jacobi", 10000, {"sym": 0}),
                                                 ("poisson2d", 256, "jacobi", 10000, {"sym": 0}),
                                                 # x step every iteration (xb = 1: the residual update
                                                 # reads r, no r0): poll not a multiple of 4, or knob 29 = 1
                                                 ("poisson3d", 128, "jacobi", 10000, {"poll": 6}),
                                                 ("poisson3d", 128, "jacobi", 10000, {"xb": 1}),
                                                 ("poisson3d", 128, "jacobi", 41, {"xb": 1}),
                                                 ("poisson3d27", 128, "jacobi", 10000, {"poll": 6}),
                                                 ("poisson2d", 256, "jacobi", 10000, {"xb": 1, "guess": True}),
                                                 ])
def test_mode5_recomputed_product(selfcomm, oracle_mod, kind, n, pc, max_it, kw):
    """CG mode 5 (knob 9 = 5): the MatMult stores no product -- a p.Ap pass
    gives p.w, and the update pass recomputes A p (the same row sums as a
    stored product, bit for bit) where it forms r - alpha A p and the norms.
    The p.Ap scalar itself is not PETSc's VecDot(p, A p) bit for bit: the
    symmetric forward-half pass sums p_i (a_ii p_i + 2 fwd_i), the same exact
    terms in another order, so the iterates match to rounding (the bars
    below).  Against the oracle: its
    and reason equal, history within 1e-8, x within rel-L2 1e-10; against mode
    2 (the stored-product iteration): the same its and reason, iterates equal
    to rounding (the norms' partials are grouped per z-march column); the
    graph-replayed second solve gives the first one's bits; the dispatch
    counts show both mode-5 passes ran.  x steps batched by 4 (the mode-5
    default) and by 2, stops at every position relative to the batch.  The
    27-point operator (knob 55) runs both passes on its column-word z-march,
    its p.Ap pass summing each row's forward half (the operator is symmetric:
    knob 59; p.Ap then equals mode 2's p.w to rounding, the bar above)."""
    from mxsolve import _lib
    from mxsolve.core import DMat, dispatch_counts, rhs_hash
    L = _lib.load()
    guess = kw.get("guess", False)
    norm = kw.get("norm", "default")

    def run(mode):
        old = L.mx_debug_set(9, mode)
        old27 = L.mx_debug_set(27, 1)           # the row-pair layout (this module's fixture turns it off)
        old29 = L.mx_debug_set(29, kw.get("xb", 0) if mode == 5 else 0)   # mode 5: x batches of 4 by default
        old59 = L.mx_debug_set(59, kw.get("sym", 1))   # 27-point: the symmetric forward-half p.Ap pass
        old60 = L.mx_debug_set(60, kw.get("k60", 1))   # 27-point: the plane-pipelined z-march
        try:
            A = DMat.stencil(selfcomm, kind, n)
            m = A.info()["m"]
            b = selfcomm.empty(m)
            rhs_hash(selfcomm, 0, b)
            x0 = selfcomm.zeros(m)
            if guess:
                rhs_hash(selfcomm, 7, x0)
                x0.mul_(0.25)
            x = selfcomm.zeros(m)
            outs = []
            dispatch_counts(reset=True)
            for k in range(2):                  # the second solve replays the cached graph
                x.copy_(x0)
                r = A.solve(b, x, ksp="cg", pc=pc, rtol=1e-8, max_it=max_it, history=True, norm=norm,
                            guess_nonzero=guess, poll_every=kw.get("poll", 16))
                if mode == 5:
                    exp_xb = 1 if (kw.get("xb") == 1 or kw.get("poll", 16) % kw.get("xb", 4)) else kw.get("xb", 4)
                    assert r["cg_mode"] == 5 and r["cg_xbatch"] == exp_xb, (r["cg_mode"], r["cg_xbatch"], exp_xb)
                outs.append((r["its"], r["reason"], r["history"].copy(), x.cpu().numpy().copy()))
                if k == 0:
                    dc = dispatch_counts(reset=True)
            A.destroy()
            return outs, dc, b.cpu().numpy(), x0.cpu().numpy()
        finally:
            L.mx_debug_set(9, old)
            L.mx_debug_set(27, old27)
            L.mx_debug_set(29, old29)
            L.mx_debug_set(59, old59)
            L.mx_debug_set(60, old60)

    m5, dc5, bh, x0 = run(5)
    m2, dc2, _, _ = run(2)
    # (a nonzero guess forms r = b - A x with the stored-product MatMult first)
    zk = "pair_zm27" if kind == "poisson3d27" else "pair_zm"
    assert dc5["zm_pw"] > 0 and dc5["zm_rupd"] > 0 and dc5[zk] == (1 if guess else 0), dc5
    assert dc2["zm_pw"] == 0 and dc2[zk] > 0, dc2
    for a, c in zip(m5, m2):
        assert a[:2] == c[:2], (a[:2], c[:2])
        assert np.allclose(a[2], c[2], rtol=1e-10, atol=0)
        assert np.linalg.norm(a[3] - c[3]) <= 1e-12 * max(np.linalg.norm(c[3]), 1e-300)
    assert m5[0][:2] == m5[1][:2]
    assert np.array_equal(m5[0][2].view(np.uint64), m5[1][2].view(np.uint64))
    assert np.array_equal(m5[0][3].view(np.uint64), m5[1][3].view(np.uint64))
    ip, c_, v = oracle_mod.stencil(kind, n)
    O = oracle_mod.OracleMat.from_csr(ip.size - 1, ip.size - 1, ip, c_, v)
    from _hostinfo import host_threads
    o = O.solve(bh, x0=x0 if guess else None, ksp="cg", pc=pc, rtol=1e-8, max_it=max_it, norm=norm, history=True,
                nthreads=host_threads())
    assert (m5[0][0], m5[0][1]) == (o["its"], o["reason"]), (m5[0][:2], o["its"], o["reason"])
    assert np.allclose(m5[0][2], o["history"], rtol=1e-8, atol=0)
    assert np.linalg.norm(m5[0][3] - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])


def test_mode5_nonsymmetric_full_rows(selfcomm, oracle_mod):
    """CG mode 5 on a constant-coefficient 7-point operator that is not
    symmetric (+D coupling -1.5, -D -1): the symmetry check (Mat::sym, once per
    operator) refuses the forward-half p.Ap pass, so the pass sums full rows
    and the solve matches the oracle (a forward-half pass would not: p.Ap of a
    nonsymmetric A is not p_i (a_ii p_i + 2 fwd_i))."""
    from mxsolve import _lib
    from mxsolve.core import DMat, dispatch_counts
    L = _lib.load()
    n = 128
    ip, c, v = oracle_mod.stencil("poisson3d", n)
    M = ip.size - 1
    rows = np.repeat(np.arange(M), np.diff(ip))
    v = np.where(c - rows == n * n, -1.5, v)
    b = np.random.default_rng(47).random(M)
    old = L.mx_debug_set(9, 5)
    old27 = L.mx_debug_set(27, 1)           # the row-pair layout (this module's fixture turns it off)
    try:
        A = DMat.from_csr(selfcomm, M, M, ip, c, v)
        assert A.info()["pair_uniform"] == 1
        x = torch.zeros(M, dtype=torch.float64, device="cuda")
        dispatch_counts(reset=True)
        r = A.solve(torch.from_numpy(b).cuda(), x, ksp="cg", pc="jacobi", rtol=1e-8, max_it=300, history=True)
        dc = dispatch_counts(reset=True)
        A.destroy()
    finally:
        L.mx_debug_set(9, old)
        L.mx_debug_set(27, old27)
    assert dc["zm_pw"] > 0 and dc["zm_rupd"] > 0, dc
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    o = O.solve(b, ksp="cg", pc="jacobi", rtol=1e-8, max_it=300, history=True)
    assert (r["its"], r["reason"]) == (o["its"], o["reason"]), (r["its"], r["reason"], o["its"], o["reason"])
    assert np.allclose(r["history"], o["history"], rtol=1e-8, atol=0)
    assert np.linalg.norm(x.cpu().numpy() - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])


def test_history_entries_not_written_read_zero(selfcomm, oracle_mod):
    """A residual-history entry that no kernel writes (the solve above stops
    at iteration 2 and PETSc's history holds 0.0 there) reads as 0.0 again
    after a GMRES solve on the same operator has filled the shared KSP work
    space -- not as that solve's leftovers (found by filling reused device
    blocks with 0xA5 bytes, knob 81 = 2)."""
    from mxsolve import _lib
    from mxsolve.core import DMat
    L = _lib.load()
    n = 128
    ip, c, v = oracle_mod.stencil("poisson3d", n)
    M = ip.size - 1
    rows = np.repeat(np.arange(M), np.diff(ip))
    v = np.where(c - rows == n * n, -1.5, v)
    b = torch.from_numpy(np.random.default_rng(47).random(M)).cuda()
    old = L.mx_debug_set(9, 5)
    old27 = L.mx_debug_set(27, 1)
    try:
        A = DMat.from_csr(selfcomm, M, M, ip, c, v)
        x = torch.zeros(M, dtype=torch.float64, device="cuda")
        r1 = A.solve(b, x, ksp="cg", pc="jacobi", rtol=1e-8, max_it=300, history=True)
        y = torch.zeros(M, dtype=torch.float64, device="cuda")
        A.solve(b, y, ksp="gmres", pc="jacobi", rtol=0.0, max_it=60)
        x.zero_()
        r3 = A.solve(b, x, ksp="cg", pc="jacobi", rtol=1e-8, max_it=300, history=True)
        A.destroy()
    finally:
        L.mx_debug_set(9, old)
        L.mx_debug_set(27, old27)
    h1, h3 = np.asarray(r1["history"]), np.asarray(r3["history"])
    assert (r1["its"], r1["reason"]) == (r3["its"], r3["reason"])
    assert np.array_equal(h1.view(np.uint64), h3.view(np.uint64)), (h1, h3)


@pytest.mark.parametrize("dims,max_it", [((128, 128, 128), 10000), ((256, 128, 40), 10000), ((128, 128, 128), 37)])
def test_two_line_residual_update(selfcomm, oracle_mod, dims, max_it):
    """Knob 68: CG mode 5's residual update with two lines per wave (line y's
    +n operand is line y + 1's own rows) sums every row exactly as the one-line
    z-march does; a wave's [z.z, z.r, r.r] partials then cover other rows than
    the one-line kernel's, so the norms -- and through them the iterates --
    equal the default's to rounding: its and reason equal, history within
    1e-10, x within 1e-12; the dispatch shows the residual update ran."""
    from mxsolve import _lib
    from mxsolve.core import DMat, dispatch_counts, rhs_hash
    L = _lib.load()
    old27 = L.mx_debug_set(27, 1)               # the row-pair layout (this module's fixture turns it off)
    try:
        A = DMat.stencil(selfcomm, "poisson3d", *dims)
    finally:
        L.mx_debug_set(27, old27)
    m = A.info()["m"]
    b = selfcomm.empty(m)
    rhs_hash(selfcomm, 0, b)
    outs = []
    for k68 in (0, 1):
        old = {k: L.mx_debug_set(k, v) for k, v in ((9, 5), (27, 1), (68, k68))}
        try:
            x = selfcomm.zeros(m)
            dispatch_counts(reset=True)
            r = A.solve(b, x, ksp="cg", pc="jacobi", rtol=1e-8, max_it=max_it, history=True)
            dc = dispatch_counts(reset=True)
            outs.append((r["its"], r["reason"], r["history"].copy(), x.cpu().numpy().copy(), r["cg_mode"], dc))
        finally:
            for k, v in old.items():
                L.mx_debug_set(k, v)
    A.destroy()
    a, c = outs
    assert a[4] == c[4] == 5 and c[5]["zm_rupd"] > 0, (a[4], c[4], c[5])
    assert a[:2] == c[:2]
    assert np.allclose(a[2], c[2], rtol=1e-10, atol=0)
    assert np.linalg.norm(a[3] - c[3]) <= 1e-12 * np.linalg.norm(a[3])


@pytest.mark.parametrize("kind,dims,pc,guess,max_it", [
    ("poisson3d", (128, 128, 128), "jacobi", False, 10000),
    ("poisson3d", (256, 128, 40), "none", False, 10000),
    ("poisson3d", (128, 128, 64), "jacobi", True, 10000),
    ("poisson3d", (128, 128, 128), "jacobi", False, 37),
    ("poisson2d", (1024, 1024, 1), "jacobi", False, 10000),
])
def test_fused_direction_pw_bitwise(selfcomm, kind, dims, pc, guess, max_it):
    """Knob 69: CG mode 5's direction update fused into the p.Ap pass forms
    every p_i operand from r_i and p_{i-1} with the direction update's own
    expression and sums p.Ap over the PW pass's units on its grid (the x-step
    batch iterations keep the separate passes): the whole solve -- its,
    reason, residual history, x -- is bitwise the separate passes' (the
    initial norms then take their own pass over b: the same bits); the
    dispatch shows the fused pass ran in place of some PW passes."""
    from mxsolve import _lib
    from mxsolve.core import DMat, dispatch_counts, rhs_hash
    L = _lib.load()
    old27 = L.mx_debug_set(27, 1)
    try:
        A = DMat.stencil(selfcomm, kind, *dims)
    finally:
        L.mx_debug_set(27, old27)
    m = A.info()["m"]
    b = selfcomm.empty(m)
    rhs_hash(selfcomm, 0, b)
    x0 = None
    if guess:
        x0 = selfcomm.empty(m)
        rhs_hash(selfcomm, 5, x0)
        x0.mul_(1e-3)
    outs = []
    for k69 in (0, 1):
        old = {k: L.mx_debug_set(k, v) for k, v in ((9, 5), (27, 1), (69, k69))}
        try:
            x = x0.clone() if guess else selfcomm.zeros(m)
            dispatch_counts(reset=True)
            r = A.solve(b, x, ksp="cg", pc=pc, rtol=1e-8, max_it=max_it, history=True, guess_nonzero=guess)
            dc = dispatch_counts(reset=True)
            outs.append((r["its"], r["reason"], r["history"].copy(), x.cpu().numpy().copy(), r["cg_mode"], dc))
        finally:
            for k, v in old.items():
                L.mx_debug_set(k, v)
    A.destroy()
    a, c = outs
    assert a[4] == c[4] == 5, (a[4], c[4])
    assert a[5]["zm_pbw"] == 0 and a[5]["zm_pw"] > 0, a[5]
    assert c[5]["zm_pbw"] > 0 and 0 < c[5]["zm_pw"] < a[5]["zm_pw"], c[5]
    assert a[:2] == c[:2]
    assert np.array_equal(a[2].view(np.uint64), c[2].view(np.uint64))
    assert np.array_equal(a[3].view(np.uint64), c[3].view(np.uint64))


@pytest.mark.parametrize("dims,max_it", [((128, 128, 16), 10000), ((256, 128, 24), 10000), ((512, 256, 16), 10000),
                                         ((128, 128, 16), 23), ((128, 3, 40), 10000)])
def test_two_line_27point(selfcomm, dims, max_it):
    """Knob 70: the 27-point plane-pipelined z-march with two lines per wave
    (line y's dy = +1 run is line y + 1's centre run, loaded once) sums every
    row exactly as the one-line kernel: the MatMult y = A x is bitwise the
    default's; CG mode 5's residual update then groups its norm partials by
    other rows, so the solve equals the default's to rounding (its and reason
    equal, history within 1e-10, x within 1e-12).  128 x 3 x 40 has an odd
    number of lines per plane: the layout does not pair and the solve is the
    default's bit for bit."""
    from mxsolve import _lib
    from mxsolve.core import DMat, dispatch_counts, rhs_hash
    L = _lib.load()
    old27 = L.mx_debug_set(27, 1)
    try:
        A = DMat.stencil(selfcomm, "poisson3d27", *dims)
    finally:
        L.mx_debug_set(27, old27)
    m = A.info()["m"]
    b = selfcomm.empty(m)
    rhs_hash(selfcomm, 0, b)
    xin = selfcomm.empty(m)
    rhs_hash(selfcomm, 3, xin)
    pairs = dims[1] % 2 == 0
    outs = []
    for k70 in (0, 1):
        old = {k: L.mx_debug_set(k, v) for k, v in ((9, 5), (27, 1), (70, k70))}
        try:
            y = selfcomm.zeros(m)
            A.mult(xin, y)
            x = selfcomm.zeros(m)
            dispatch_counts(reset=True)
            r = A.solve(b, x, ksp="cg", pc="jacobi", rtol=1e-8, max_it=max_it, history=True)
            dc = dispatch_counts(reset=True)
            outs.append((r["its"], r["reason"], r["history"].copy(), x.cpu().numpy().copy(), r["cg_mode"], dc,
                         y.cpu().numpy().copy()))
        finally:
            for k, v in old.items():
                L.mx_debug_set(k, v)
    A.destroy()
    a, c = outs
    assert np.array_equal(a[6].view(np.uint64), c[6].view(np.uint64))
    assert a[:2] == c[:2]
    if not pairs:                               # (not the column-word layout: mode 2 here)
        assert a[4] == c[4] and a[5] == c[5]
        assert np.array_equal(a[2].view(np.uint64), c[2].view(np.uint64))
        assert np.array_equal(a[3].view(np.uint64), c[3].view(np.uint64))
        return
    assert a[4] == c[4] == 5 and c[5]["zm_rupd"] > 0, (a[4], c[4], c[5])
    assert np.allclose(a[2], c[2], rtol=1e-10, atol=0)
    assert np.linalg.norm(a[3] - c[3]) <= 1e-12 * np.linalg.norm(a[3])


@pytest.mark.parametrize("kind,dims,mode,max_it", [
    ("poisson3d", (256, 128, 40), 5, 10000), ("poisson3d", (256, 128, 40), 5, 37), ("poisson3d", (256, 128, 40), 5, 20),
    ("poisson3d", (128, 128, 128), 5, 10000), ("poisson3d", (256, 128, 40), 2, 10000), ("poisson3d", (256, 128, 40), 2, 29),
    ("poisson3d27", (128, 128, 16), 5, 10000), ("poisson2d", (1024, 1024, 1), 5, 10000),
])
def test_xbatch8_bitwise(selfcomm, kind, dims, mode, max_it):
    """Knob 29 = 8: x steps batched by eight (eight direction buffers) apply
    the same fma(a_j, p_j, x) chain oldest first as batches of four -- x never
    feeds back into the iteration -- so the whole solve (its, reason, history,
    x) is bitwise the same; max_it 37 / 20 / 29 stop with 5 / 4 / 5 steps
    pending for the finish pass."""
    from mxsolve import _lib
    from mxsolve.core import DMat, rhs_hash
    L = _lib.load()
    old27 = L.mx_debug_set(27, 1)
    try:
        A = DMat.stencil(selfcomm, kind, *dims)
    finally:
        L.mx_debug_set(27, old27)
    m = A.info()["m"]
    b = selfcomm.empty(m)
    rhs_hash(selfcomm, 0, b)
    outs = []
    for xb in (4, 8):
        old = {k: L.mx_debug_set(k, v) for k, v in ((9, mode), (27, 1), (29, xb))}
        try:
            x = selfcomm.zeros(m)
            r = A.solve(b, x, ksp="cg", pc="jacobi", rtol=1e-8, max_it=max_it, history=True)
            outs.append((r["its"], r["reason"], r["history"].copy(), x.cpu().numpy().copy(), r["cg_mode"],
                         r["cg_xbatch"]))
        finally:
            for k, v in old.items():
                L.mx_debug_set(k, v)
    A.destroy()
    a, c = outs
    assert a[4] == c[4] == mode and (a[5], c[5]) == (4, 8), (a[4:], c[4:])
    assert a[:2] == c[:2]
    assert np.array_equal(a[2].view(np.uint64), c[2].view(np.uint64))
    assert np.array_equal(a[3].view(np.uint64), c[3].view(np.uint64))


@pytest.mark.parametrize("max_it", [20, 37, 10000])
def test_finish_unaligned_x(selfcomm, max_it):
    """The batched x steps' finish pass takes 16-byte row pairs when the
    caller's x is 16-byte aligned and one row per step otherwise (an x that
    is a view one element into a larger buffer): the same bits either way."""
    from mxsolve import _lib
    from mxsolve.core import DMat, rhs_hash
    L = _lib.load()
    old27 = L.mx_debug_set(27, 1)
    try:
        A = DMat.stencil(selfcomm, "poisson3d", 128, 128, 40)
    finally:
        L.mx_debug_set(27, old27)
    m = A.info()["m"]
    b = selfcomm.empty(m)
    rhs_hash(selfcomm, 0, b)
    xa = selfcomm.zeros(m)
    big = selfcomm.zeros(m + 1)
    xu = big[1:]
    assert xu.data_ptr() % 16 == 8
    ra = A.solve(b, xa, ksp="cg", pc="jacobi", rtol=1e-8, max_it=max_it)
    ru = A.solve(b, xu, ksp="cg", pc="jacobi", rtol=1e-8, max_it=max_it)
    A.destroy()
    assert (ra["its"], ra["reason"]) == (ru["its"], ru["reason"])
    assert torch.equal(xa.view(torch.int64), xu.contiguous().view(torch.int64))
