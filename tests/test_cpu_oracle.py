"""Pin the oracle (C restatement of PETSc, oracle/petsc_oracle.c) against the
reference's own fixtures and known answers before trusting it as the checker."""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def meta():
    with open(os.path.join(HERE, "golden", "reference_systems.json")) as f:
        return json.load(f)


def test_fixture_hashes(golden, meta):
    import hashlib
    for k, v in meta["sha12"].items():
        assert hashlib.sha256(np.ascontiguousarray(golden[k]).tobytes()).hexdigest()[:12] == v, k
    # SURVEY Appendix B values computed from the reference's create_system
    assert meta["sha12"]["sys_indptr"] == "19e20173b4b8"
    assert meta["sha12"]["sys_B"] == "87a74ab59e1d"


def test_split_ownership_matches_driver(oracle_mod, meta):
    """PetscSplitOwnership == the driver's divmod split (test.py:68-74)."""
    for P, d in meta["splits"].items():
        r = oracle_mod.split_ownership(100, int(P))
        assert list(np.diff(r)) == d["count"] and list(r[:-1]) == d["displ"]


def test_assembly_identity_on_reference_inputs(oracle_mod, golden):
    """The reference's CSR inputs are canonical, so MatGetRow returns them byte-for-byte."""
    for pre, n in (("sys", 100), ("tri", 100)):
        for P in (1, 2, 3, 4):
            A = oracle_mod.OracleMat.from_csr(n, n, golden[f"{pre}_indptr"], golden[f"{pre}_indices"],
                                              golden[f"{pre}_data"], P=P)
            ip, c, v = A.csr()
            assert np.array_equal(ip, golden[f"{pre}_indptr"]) and np.array_equal(c, golden[f"{pre}_indices"])
            assert np.array_equal(v, golden[f"{pre}_data"])


def test_mpiaij_split_counts(oracle_mod, golden):
    """P=2 -> rank0 239 diag/243 offdiag/50 ghosts, rank1 277/241/50;
    P=4 ghosts 70/70/68/70; tridiagonal P=2 -> 148 diag + 1 offdiag per rank."""
    A = oracle_mod.OracleMat.from_csr(100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"], P=2)
    b0, b1 = A.block(0), A.block(1)
    assert (len(b0["dval"]), len(b0["oval"]), len(b0["garray"])) == (239, 243, 50)
    assert (len(b1["dval"]), len(b1["oval"]), len(b1["garray"])) == (277, 241, 50)
    A4 = oracle_mod.OracleMat.from_csr(100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"], P=4)
    assert [len(A4.block(r)["garray"]) for r in range(4)] == [70, 70, 68, 70]
    T = oracle_mod.OracleMat.from_csr(100, 100, golden["tri_indptr"], golden["tri_indices"], golden["tri_data"], P=2)
    assert [(len(T.block(r)["dval"]), len(T.block(r)["oval"])) for r in range(2)] == [(148, 1), (148, 1)]


def test_garray_sorted_and_remap(oracle_mod, golden):
    A = oracle_mod.OracleMat.from_csr(100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"], P=3)
    for r in range(3):
        b = A.block(r)
        g = b["garray"]
        assert np.all(np.diff(g) > 0)
        assert b["ocol"].size == 0 or b["ocol"].max() < g.size


def test_insert_and_add_semantics(oracle_mod):
    """MatSetValues: negative columns ignored, INSERT keeps the last duplicate, ADD sums in order."""
    ip = np.array([0, 5, 7])
    cols = np.array([3, 1, -1, 3, 0, 2, 2])
    vals = np.array([1.0, 2.0, 9.0, 4.0, 5.0, 0.0, 7.0])
    A = oracle_mod.OracleMat.from_csr(2, 4, ip, cols, vals)
    assert [list(a) for a in A.csr()] == [[0, 3, 4], [0, 1, 3, 2], [5.0, 2.0, 4.0, 7.0]]
    B = oracle_mod.OracleMat.from_csr(2, 4, ip, cols, vals, add=True)
    assert list(B.csr()[2]) == [5.0, 2.0, 5.0, 7.0]
    with pytest.raises(ValueError):
        oracle_mod.OracleMat.from_csr(2, 4, ip, np.array([3, 1, 4, 3, 0, 2, 2]), vals)


def test_stash_order(oracle_mod):
    """Off-process MatSetValues: the owner applies its own entries first, then
    the stashed ones by source rank; the assembled sum matches scipy's."""
    per_rank = [(np.array([3, 0, 4]), np.array([0, 0, 1]), np.array([1.0, 2.0, 3.0])),
                (np.array([0, 3, -1]), np.array([0, 0, 2]), np.array([10.0, 20.0, 99.0])),
                (np.array([0]), np.array([1]), np.array([5.0]))]
    ptr, r, c, v = oracle_mod.stash_order(5, 3, per_rank)   # ranges 0,2,4,5
    assert list(ptr) == [0, 3, 5, 6]
    assert list(zip(r, c, v)) == [(0, 0, 2.0), (0, 0, 10.0), (0, 1, 5.0), (3, 0, 20.0), (3, 0, 1.0), (4, 1, 3.0)]
    A = oracle_mod.OracleMat.from_coo(5, 5, ptr, r, c, v, P=3, add=True)
    I = oracle_mod.OracleMat.from_coo(5, 5, ptr, r, c, v, P=3, add=False)
    ip, cj, vv = A.csr()
    assert list(cj) == [0, 1, 0, 1] and list(vv) == [12.0, 5.0, 21.0, 3.0]
    assert list(I.csr()[2]) == [10.0, 5.0, 1.0, 3.0]   # row 3: owner rank 1's 20, then rank 0's 1


def test_spmv_matches_scipy(oracle_mod, golden):
    S = sp.csr_matrix((golden["sys_data"], golden["sys_indices"], golden["sys_indptr"]), shape=(100, 100))
    A = oracle_mod.OracleMat.from_csr(100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"], P=3)
    x = np.random.default_rng(0).standard_normal(100)
    assert np.allclose(A.mult(x), S @ x, rtol=1e-14, atol=1e-14)
    assert np.allclose(A.mult(golden["sys_X"]), golden["sys_B"], rtol=1e-13, atol=1e-14)


def test_stencil_nnz_formulas(oracle_mod):
    """nnz(2D 5-pt) = 5n^2-4n, nnz(3D 7-pt) = 7n^3-6n^2, nnz(27-pt) = (3n-2)^3."""
    for n in (3, 7, 10):
        assert oracle_mod.stencil("poisson2d", n)[1].size == 5 * n * n - 4 * n
        assert oracle_mod.stencil("poisson3d", n)[1].size == 7 * n**3 - 6 * n**2
        assert oracle_mod.stencil("poisson3d27", n)[1].size == (3 * n - 2) ** 3


def test_convdiff_properties(oracle_mod):
    ip, c, v = oracle_mod.stencil("convdiff3d", 9)
    S = sp.csr_matrix((v, c, ip))
    assert np.all(np.mod(v * 4, 1) == 0)                 # dyadic, multiples of 1/4
    assert abs(S - S.T).max() == 0.5                      # nonsymmetric by the upwind term


def test_rhs_hash_known_values(oracle_mod):
    b = oracle_mod.rhs_hash(0, 4)
    assert np.all((b >= 0) & (b < 1))
    b2 = oracle_mod.rhs_hash(2, 2)
    assert np.array_equal(b[2:], b2)                      # partition independent


def test_cg_known_answers(oracle_mod):
    """Jacobi-PCG iteration counts (3D 7-pt 32^3 = 84) and the true residual."""
    ip, c, v = oracle_mod.stencil("poisson3d", 32)
    M = ip.size - 1
    A = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    b = oracle_mod.rhs_hash(0, M)
    r = A.solve(b, ksp="cg")
    assert (r["its"], r["reason"]) == (84, 2)
    S = sp.csr_matrix((v, c, ip))
    assert np.linalg.norm(S @ r["x"] - b) / np.linalg.norm(b) < 1e-4
    # P-rank restatement: same iteration count, rounding-level difference only
    r4 = oracle_mod.OracleMat.from_csr(M, M, ip, c, v, P=4).solve(b, ksp="cg")
    assert r4["its"] == 84 and np.linalg.norm(r4["x"] - r["x"]) / np.linalg.norm(r["x"]) < 1e-12


def test_gmres_known_answers(oracle_mod, golden):
    """Conv-diff 16^3 GMRES(30)+Jacobi = 55 its (SURVEY cdprobe); test.py system with
    GMRES(100)+Jacobi recovers X_actual (test.py:149's check)."""
    ip, c, v = oracle_mod.stencil("convdiff3d", 16)
    M = ip.size - 1
    r = oracle_mod.OracleMat.from_csr(M, M, ip, c, v).solve(oracle_mod.rhs_hash(0, M), ksp="gmres")
    assert (r["its"], r["reason"]) == (55, 2)
    A = oracle_mod.OracleMat.from_csr(100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"])
    g = A.solve(golden["sys_B"], ksp="gmres", restart=100, max_it=1000)
    assert g["reason"] == 2 and np.allclose(g["x"], golden["sys_X"])
    # CG on the indefinite nonsymmetric test.py matrix does not converge
    cg = A.solve(golden["sys_B"], ksp="cg", max_it=2000)
    assert cg["reason"] < 0


def test_convergence_reasons(oracle_mod):
    ip, c, v = oracle_mod.stencil("poisson3d", 8)
    M = ip.size - 1
    A = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    assert A.solve(np.zeros(M), ksp="cg")["reason"] == 3          # CONVERGED_ATOL on zero rhs
    assert A.solve(np.ones(M), ksp="cg", max_it=3)["reason"] == -3  # DIVERGED_ITS
    r = A.solve(np.ones(M), ksp="cg", norm="none", max_it=5)
    assert (r["its"], r["reason"]) == (5, 4)                        # KSPConvergedSkip -> CONVERGED_ITS
    ind = oracle_mod.OracleMat.from_csr(2, 2, np.array([0, 1, 2]), np.array([0, 1]), np.array([1.0, -1.0]))
    assert ind.solve(np.ones(2), ksp="cg", pc="none")["reason"] == -10    # p.Ap == 0: DIVERGED_INDEFINITE_MAT
    assert A.solve(np.ones(M), ksp="preonly")["its"] == 1


def test_oracle_maxpy_grouping(oracle_mod):
    """The oracle's VecMAXPY_Seq restatement: the first nv % 4 vectors, then
    groups of four, each summed left to right before it is added to y."""
    import numpy as np
    rng = np.random.default_rng(3)
    for nv in (1, 2, 3, 4, 5, 6, 9):
        xs = [rng.standard_normal(257) for _ in range(nv)]
        y = rng.standard_normal(257)
        a = rng.standard_normal(nv)
        u = y.copy()
        r = nv % 4
        if r == 1:
            u = a[0] * xs[0] + u
        elif r == 2:
            u = u + (a[0] * xs[0] + a[1] * xs[1])
        elif r == 3:
            u = u + ((a[0] * xs[0] + a[1] * xs[1]) + a[2] * xs[2])
        for j in range(r, nv, 4):
            u = u + (((a[j] * xs[j] + a[j + 1] * xs[j + 1]) + a[j + 2] * xs[j + 2]) + a[j + 3] * xs[j + 3])
        assert np.array_equal(oracle_mod.vec_maxpy(y, a, xs), u)


def test_bench_host_csr_equals_oracle_stencil(oracle_mod):
    """bench.py builds test.py-style host CSR arrays (int32 I/J, fp64 V) with
    numpy for its createAIJ-from-host leg: the same matrices as the oracle's
    stencil generator (7-point and 27-point, non-cubic grids)."""
    import bench
    for kind, okind, dims in (("7pt", "poisson3d", (6, 5, 4)), ("27pt", "poisson3d27", (5, 4, 3)),
                              ("7pt", "poisson3d", (16, 16, 16))):
        ip, c, v = bench.host_csr_stencil(*dims, kind)
        oi, oc, ov = oracle_mod.stencil(okind, *dims)
        assert ip.dtype == np.int32 and c.dtype == np.int32
        assert np.array_equal(ip, oi) and np.array_equal(c, oc) and np.array_equal(v.view(np.uint64), ov.view(np.uint64))


def test_bench_general_leg_checker(oracle_mod):
    """bench.py's spmv_general leg: the variable-coefficient 7-point operator
    (canonical CSR: ascending columns, 7n^3 - 6n^2 entries, symmetric, diagonal
    = the sum of the face kappas) and the row-ordered product it checks the
    GPU MatMult against, which must equal the oracle's MatMult_SeqAIJ bit for
    bit (the checker cannot be weaker than the oracle)."""
    import bench
    n = 12
    N, ip, c, v = bench.varcoef_csr(n)
    assert N == n ** 3 and ip[-1] == 7 * n ** 3 - 6 * n ** 2
    assert all(np.all(np.diff(c[ip[i]:ip[i + 1]]) > 0) for i in range(N))
    import scipy.sparse as sp
    A = sp.csr_matrix((v, c, ip), shape=(N, N))
    assert abs(A - A.T).max() == 0.0
    d = A.diagonal()
    assert len(np.unique(v)) > 2 * N and np.all(d > 0)
    O = oracle_mod.OracleMat.from_csr(N, N, ip, c, v)
    for seed in range(3):
        x = np.random.default_rng(seed).standard_normal(N)
        got = bench.csr_rowsum_reference(ip, c, v, x)
        assert np.array_equal(got.view(np.uint64), O.mult(x).view(np.uint64))


def test_bench_parity_record():
    """bench.py's parity block: ok only with equal its, equal reason and
    rel-L2 <= 1e-10."""
    import bench
    o = {"its": 560, "reason": 2, "P": 1, "solve_s": 1.0}
    assert bench.parity_record(560, 2, 3e-14, o)["ok"]
    assert not bench.parity_record(561, 2, 3e-14, o)["ok"]
    assert not bench.parity_record(560, 3, 3e-14, o)["ok"]
    assert not bench.parity_record(560, 2, 2e-10, o)["ok"]


def test_bench_choose_leg():
    """bench.py takes value from the fastest parity-passing leg; a faster leg
    that failed parity is never chosen; with no passing leg, the first."""
    import bench
    legs = [{"leg": "a", "value": 10.0, "parity": {"ok": True}},
            {"leg": "b", "value": 30.0, "parity": {"ok": False}},
            {"leg": "c", "value": 20.0, "parity": {"ok": True}}]
    assert bench.choose_leg(legs)["leg"] == "c"
    assert bench.choose_leg([dict(l, parity={"ok": False}) for l in legs])["leg"] == "a"
    assert bench.choose_leg([{"leg": "x", "value": 1.0}, {"leg": "y", "value": 2.0}], no_solve=True)["leg"] == "y"
    assert bench.rnd(None, 3) is None and bench.rnd(1.23456, 2) == 1.23
