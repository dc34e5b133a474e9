"""The column-block two-pass MatMult (mx_spmv_cb.hip) for unstructured AIJ
blocks -- test.py:14's scipy.sparse.random family.  Bar: MatMult bit-exact
against the oracle's MatMult_SeqAIJ restatement and against the one-pass SELL
kernel (key 84 = 0); GMRES(30) + Jacobi through it bit for bit the one-pass
run, with its and reason equal to the oracle's and x within relative L2
1e-10; the auto choice takes random patterns of >= 2^20 rows and leaves
stencils alone."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _random_csr(N, k, seed, ragged=False):
    """Rows of k random columns (the diagonal included, no repeats, ascending);
    ragged: 0..2k entries per row, empty rows included."""
    rng = np.random.default_rng(seed)
    ip = [0]
    cols, vals = [], []
    for r in range(N):
        n = int(rng.integers(0, 2 * k + 1)) if ragged else k
        c = set(rng.integers(0, N, size=max(n - 1, 0)).tolist()) | ({r} if n else set())
        c = sorted(c)
        v = -rng.random(len(c))
        for j, cc in enumerate(c):
            if cc == r:
                v[j] = 1.0 + np.abs(v).sum()
        cols += c
        vals += v.tolist()
        ip.append(len(cols))
    return np.array(ip, np.int64), np.array(cols, np.int32), np.array(vals)


def _knob(k, v):
    from mxsolve import _lib
    return _lib.load().mx_debug_set(k, v)


def _mat(comm, N, ip, c, v, cb):
    from mxsolve.core import DMat
    old = _knob(84, cb)
    try:
        return DMat.from_csr(comm, N, N, ip, c, v)
    finally:
        _knob(84, old)


@pytest.mark.parametrize("ragged", [False, True])
def test_cb_matmult_bitexact(selfcomm, oracle_mod, ragged):
    from mxsolve.core import dispatch_counts
    N = 1 << 14 if not ragged else 6000
    ip, c, v = _random_csr(N, 7, 3 + ragged, ragged)
    A = _mat(selfcomm, N, ip, c, v, 2)
    B = _mat(selfcomm, N, ip, c, v, 0)
    assert A.info()["cb_blocks"] > 0 and B.info()["cb_blocks"] == 0
    xh = np.random.default_rng(9).standard_normal(N)
    x = torch.from_numpy(xh).cuda()
    y, z = selfcomm.empty(N), selfcomm.empty(N)
    dispatch_counts(reset=True)
    A.mult(x, y)
    assert dispatch_counts()["cb"] == 1
    B.mult(x, z)
    yo = oracle_mod.OracleMat.from_csr(N, N, ip, c, v).mult(xh)
    assert np.array_equal(y.cpu().numpy().view(np.uint64), yo.view(np.uint64))
    assert np.array_equal(y.cpu().numpy().view(np.uint64), z.cpu().numpy().view(np.uint64))
    A.destroy()
    B.destroy()


def test_cb_gmres_equals_one_pass_and_oracle(selfcomm, oracle_mod):
    """GMRES(30) + Jacobi reads the operand scaled (VecScale folded into the
    MatMult) with the Jacobi fused: the two-pass MatMult keeps every bit."""
    N = 1 << 13
    ip, c, v = _random_csr(N, 7, 11)
    b = np.random.default_rng(4).random(N)
    out = {}
    for cb in (2, 0):
        A = _mat(selfcomm, N, ip, c, v, cb)
        x = selfcomm.zeros(N)
        r = A.solve(torch.from_numpy(b).cuda(), x, ksp="gmres", pc="jacobi", history=True)
        out[cb] = (r["its"], r["reason"], r["history"], x.cpu().numpy())
        A.destroy()
    a, z = out[2], out[0]
    assert (a[0], a[1]) == (z[0], z[1])
    assert np.array_equal(a[2].view(np.uint64), z[2].view(np.uint64))
    assert np.array_equal(a[3].view(np.uint64), z[3].view(np.uint64))
    o = oracle_mod.OracleMat.from_csr(N, N, ip, c, v).solve(b, ksp="gmres", pc="jacobi")
    assert (a[0], a[1]) == (o["its"], o["reason"])
    assert np.linalg.norm(a[3] - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])


def test_cb_cg_symmetric_random(selfcomm, oracle_mod):
    """CG + Jacobi on a symmetric random pattern (A + A^T + diagonal
    dominance), CG mode 2 (auto's choice from 3M rows; mode 1 fuses the
    direction update into a MatMult form the two-pass kernel does not take):
    the MatMult's p.Ap partials come from the two-pass kernel."""
    import scipy.sparse as sp
    N = 1 << 13
    ip, c, v = _random_csr(N, 5, 17)
    R = sp.csr_matrix((v, c, ip), shape=(N, N))
    S = (R + R.T).tocsr()
    S.setdiag(0.0)
    S.eliminate_zeros()
    S = S + sp.diags(1.0 + np.asarray(abs(S).sum(axis=1)).ravel())
    S = S.tocsr()
    S.sort_indices()
    b = np.random.default_rng(6).random(N)
    from mxsolve.core import dispatch_counts
    A = _mat(selfcomm, N, S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data, 2)
    assert A.info()["cb_blocks"] > 0
    x = selfcomm.zeros(N)
    old = _knob(9, 2)          # CG mode 2 (auto's choice from 3M rows): a plain MatMult + p.w
    try:
        dispatch_counts(reset=True)
        r = A.solve(torch.from_numpy(b).cuda(), x, ksp="cg", pc="jacobi")
        dc = dispatch_counts(reset=True)
    finally:
        _knob(9, old)
    assert dc["cb"] >= r["its"], dc
    o = oracle_mod.OracleMat.from_csr(N, N, S.indptr, S.indices, S.data).solve(b, ksp="cg", pc="jacobi")
    assert (r["its"], r["reason"]) == (o["its"], o["reason"])
    xv = x.cpu().numpy()
    assert np.linalg.norm(xv - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])
    A.destroy()


def test_cb_auto_choice(selfcomm):
    """Key 84 = 1 (default): a 2^20-row random pattern gets the column-block
    layout, a stencil of the same size does not; the large product is
    bit-exact against the row-ordered sum (bench.py's checker)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from mxsolve.core import DMat
    N = 1 << 20
    ip, c, v = bench.random_csr(N)
    A = DMat.from_csr(selfcomm, N, N, ip, c, v)
    assert A.info()["cb_blocks"] > 0
    xh = np.random.default_rng(2).standard_normal(N)
    y = selfcomm.empty(N)
    A.mult(torch.from_numpy(xh).cuda(), y)
    yref = bench.csr_rowsum_reference(ip, c, v, xh)
    assert np.array_equal(y.cpu().numpy().view(np.uint64), yref.view(np.uint64))
    A.destroy()
    S = DMat.stencil(selfcomm, "poisson3d", 128, 128, 64)
    assert S.info()["cb_blocks"] == 0
    S.destroy()


@pytest.mark.parametrize("P", [2, 3])
def test_cb_ranks_split(oracle_mod, P):
    """P in-process ranks: each rank's diagonal block takes the column-block
    MatMult, the rows with ghost entries are finished by the halo-boundary
    kernel.  MatMult bit-exact against the oracle; GMRES(30) + Jacobi bit for
    bit the one-pass run (key 84 = 0), its and reason the oracle's."""
    from mxsolve.core import LocalWorld, DMat
    N = 1 << 12
    ip, c, v = _random_csr(N, 7, 23)
    ranges = oracle_mod.split_ownership(N, P)
    xh = np.random.default_rng(8).standard_normal(N)
    b = np.random.default_rng(4).random(N)
    # MatMult_MPIAIJ order: the diagonal block's sum, then the ghost block's
    O = oracle_mod.OracleMat.from_csr(N, N, ip, c, v, P=P)
    yo = O.mult(xh)

    def body(comm):
        r0, r1 = ranges[comm.rank], ranges[comm.rank + 1]
        lip = ip[r0:r1 + 1] - ip[r0]
        A = DMat.from_csr(comm, N, N, lip, c[ip[r0]:ip[r1]], v[ip[r0]:ip[r1]])
        cbk = A.info()["cb_blocks"]
        y = comm.empty(r1 - r0)
        A.mult(torch.from_numpy(xh[r0:r1].copy()).cuda(), y)
        x = comm.zeros(r1 - r0)
        res = A.solve(torch.from_numpy(b[r0:r1].copy()).cuda(), x, ksp="gmres", pc="jacobi", history=True)
        A.destroy()
        return cbk, y.cpu().numpy(), res["its"], res["reason"], res["history"], x.cpu().numpy()

    outs = {}
    for cb in (2, 0):
        old = _knob(84, cb)           # set once, outside the rank threads
        w = LocalWorld(P)
        try:
            outs[cb] = w.run(body)
        finally:
            _knob(84, old)
            w.destroy()
    assert all(o[0] > 0 for o in outs[2]) and all(o[0] == 0 for o in outs[0])
    y = np.concatenate([o[1] for o in outs[2]])
    assert np.array_equal(y.view(np.uint64), yo.view(np.uint64))
    for a, z in zip(outs[2], outs[0]):
        assert (a[2], a[3]) == (z[2], z[3])
        assert np.array_equal(a[4].view(np.uint64), z[4].view(np.uint64))
        assert np.array_equal(a[5].view(np.uint64), z[5].view(np.uint64))
    o = O.solve(b, ksp="gmres", pc="jacobi")
    x = np.concatenate([a[5] for a in outs[2]])
    assert (outs[2][0][2], outs[2][0][3]) == (o["its"], o["reason"])
    assert np.linalg.norm(x - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])


def test_cb_rows_without_diagonal(selfcomm, oracle_mod):
    """Rows that hold entries but no diagonal, and explicit zeros on the
    diagonal: the pass-2 diagonal products only where a diagonal entry is."""
    N = 1 << 12
    ip, c, v = _random_csr(N, 6, 31)
    keep = np.ones(c.size, bool)
    rows = np.repeat(np.arange(N), np.diff(ip))
    keep[(c == rows) & (rows % 5 == 0)] = False        # every fifth row loses its diagonal
    v = v.copy()
    v[(c == rows) & (rows % 7 == 0)] = 0.0             # an explicit zero diagonal
    c2, v2 = c[keep], v[keep]
    ip2 = np.zeros(N + 1, np.int64)
    np.cumsum(np.bincount(rows[keep], minlength=N), out=ip2[1:])
    A = _mat(selfcomm, N, ip2, c2, v2, 2)
    assert A.info()["cb_blocks"] > 0
    xh = np.random.default_rng(12).standard_normal(N)
    y = selfcomm.empty(N)
    A.mult(torch.from_numpy(xh).cuda(), y)
    yo = oracle_mod.OracleMat.from_csr(N, N, ip2, c2, v2).mult(xh)
    assert np.array_equal(y.cpu().numpy().view(np.uint64), yo.view(np.uint64))
    A.destroy()


def test_cb_ranks_cg_split(oracle_mod):
    """CG + Jacobi (mode 2) on a symmetric random pattern over two in-process
    ranks: the MatMult's DOT form through the column-block path in split mode (the
    rows with ghost entries leave their p.y terms to the halo-boundary
    kernel).  Bit for bit the one-pass run (key 84 = 0); its and reason the
    P-rank oracle's, x within relative L2 1e-10."""
    import scipy.sparse as sp
    from mxsolve.core import LocalWorld, DMat, dispatch_counts
    P, N = 2, 1 << 13
    ip, c, v = _random_csr(N, 5, 29)
    R = sp.csr_matrix((v, c, ip), shape=(N, N))
    S = (R + R.T).tocsr()
    S.setdiag(0.0)
    S.eliminate_zeros()
    S = (S + sp.diags(1.0 + np.asarray(abs(S).sum(axis=1)).ravel())).tocsr()
    S.sort_indices()
    ip, c, v = S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data
    ranges = oracle_mod.split_ownership(N, P)
    b = np.random.default_rng(7).random(N)

    def body(comm):
        r0, r1 = ranges[comm.rank], ranges[comm.rank + 1]
        A = DMat.from_csr(comm, N, N, ip[r0:r1 + 1] - ip[r0], c[ip[r0]:ip[r1]], v[ip[r0]:ip[r1]])
        cbk = A.info()["cb_blocks"]
        x = comm.zeros(r1 - r0)
        res = A.solve(torch.from_numpy(b[r0:r1].copy()).cuda(), x, ksp="cg", pc="jacobi", history=True)
        A.destroy()
        return cbk, res["its"], res["reason"], res["history"], x.cpu().numpy()

    outs, dcs = {}, {}
    for cb in (2, 0):
        old, oldm = _knob(84, cb), _knob(9, 2)   # CG mode 2: the plain DOT MatMult
        w = LocalWorld(P)
        try:
            dispatch_counts(reset=True)
            outs[cb] = w.run(body)
            dcs[cb] = dispatch_counts(reset=True)
        finally:
            _knob(84, old)
            _knob(9, oldm)
            w.destroy()
    assert all(o[0] > 0 for o in outs[2]) and all(o[0] == 0 for o in outs[0])
    assert dcs[2]["cb"] >= P * outs[2][0][1] and dcs[0]["cb"] == 0, (dcs[2], dcs[0])
    for a, z in zip(outs[2], outs[0]):
        assert (a[1], a[2]) == (z[1], z[2])
        assert np.array_equal(a[3].view(np.uint64), z[3].view(np.uint64))
        assert np.array_equal(a[4].view(np.uint64), z[4].view(np.uint64))
    o = oracle_mod.OracleMat.from_csr(N, N, ip, c, v, P=P).solve(b, ksp="cg", pc="jacobi")
    x = np.concatenate([a[4] for a in outs[2]])
    assert (outs[2][0][1], outs[2][0][2]) == (o["its"], o["reason"])
    assert np.linalg.norm(x - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])
