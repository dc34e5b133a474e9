"""GPU parity of the hot path against the oracle (C restatement of PETSc).

Bar: assembly and SpMV bit-exact; KSP iteration counts equal and the fp64
solution within relative L2 1e-10 (north_star).  All calls go through the C ABI.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REL_TOL = 1e-10


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()


def assert_csr_equal(got, exp):
    for g, e, name in zip(got, exp, ("indptr", "cols", "vals")):
        assert g.shape == e.shape, name
        if name == "vals":
            assert np.array_equal(g.view(np.uint64), e.view(np.uint64)), name
        else:
            assert np.array_equal(g, e), name


def test_assembly_reference_system(selfcomm, golden):
    """test.py's seed-42 CSR (canonical) comes back byte-identical (MatGetRow)."""
    from mxsolve.core import DMat
    A = DMat.from_csr(selfcomm, 100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"])
    ip, c, v = A.csr()
    assert_csr_equal((ip, c, v), (golden["sys_indptr"].astype(np.int64),
                                  golden["sys_indices"].astype(np.int64), golden["sys_data"]))
    d = torch.zeros(100, dtype=torch.float64, device="cuda")
    A.diagonal(d)
    S = np.zeros(100)
    for i in range(100):
        for k in range(golden["sys_indptr"][i], golden["sys_indptr"][i + 1]):
            if golden["sys_indices"][k] == i:
                S[i] = golden["sys_data"][k]
    assert np.array_equal(d.cpu().numpy(), S)


@pytest.mark.parametrize("add", [False, True])
@pytest.mark.parametrize("maxlen", [5, 12, 40, 64, 300, 2048])
def test_assembly_unsorted_duplicates(selfcomm, oracle_mod, add, maxlen):
    """MatSetValues semantics: unsorted rows, duplicate columns, negative ids, zeros."""
    from mxsolve.core import DMat
    rng = np.random.default_rng(maxlen + 7 * add)
    M, N = 257, 300
    lens = rng.integers(0, maxlen + 1, M)
    lens[rng.integers(0, M)] = maxlen
    ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nnz = int(ip[-1])
    cols = rng.integers(-3, min(N, max(8, maxlen // 2)), nnz).astype(np.int64)
    vals = rng.standard_normal(nnz)
    vals[rng.random(nnz) < 0.05] = 0.0
    A = DMat.from_csr(selfcomm, M, N, ip, cols, vals, add=add)
    O = oracle_mod.OracleMat.from_csr(M, N, ip, cols, vals, P=1, add=add)
    assert_csr_equal(A.csr(), O.csr())


@pytest.mark.parametrize("fused", [1, 0])
@pytest.mark.parametrize("where", ["host", "device"])
@pytest.mark.parametrize("itype", [np.int32, np.int64])
@pytest.mark.parametrize("maxlen", [12, 64, 300])
def test_assembly_index_widths(selfcomm, oracle_mod, maxlen, itype, where, fused):
    """createAIJ(csr=...) with 32-bit (scipy's default) or 64-bit index arrays,
    from host arrays or device tensors: 32-bit columns are read as is by the
    fused passes and widened for the separate ones (long rows, knob 72 = 0);
    device arrays are read in place.  Same CSR as the oracle either way, and
    the column range check still fires."""
    from mxsolve import _lib
    from mxsolve._lib import MxError
    from mxsolve.core import DMat
    L = _lib.load()
    rng = np.random.default_rng(maxlen + (itype == np.int32))
    M, N = 301, 400
    lens = rng.integers(0, maxlen + 1, M)
    lens[rng.integers(0, M)] = maxlen
    ip = np.concatenate([[0], np.cumsum(lens)]).astype(itype)
    nnz = int(ip[-1])
    cols = rng.integers(-2, N, nnz).astype(itype)
    cols[: nnz // 3] = rng.integers(-1, 20, nnz // 3)     # duplicates
    vals = rng.standard_normal(nnz)
    tdt = torch.int32 if itype == np.int32 else torch.int64

    def args(c):
        if where == "host":
            return ip, c, vals
        return (torch.from_numpy(ip).to(tdt).cuda(), torch.from_numpy(c).to(tdt).cuda(), to_dev(vals))
    old = L.mx_debug_set(72, fused)
    try:
        for add in (False, True):
            A = DMat.from_csr(selfcomm, M, N, *args(cols), add=add)
            O = oracle_mod.OracleMat.from_csr(M, N, ip.astype(np.int64), cols.astype(np.int64), vals, P=1, add=add)
            assert_csr_equal(A.csr(), O.csr())
        bad = cols.copy()
        bad[nnz // 2] = N
        with pytest.raises(MxError) as e:
            DMat.from_csr(selfcomm, M, N, *args(bad))
        assert e.value.code == 2
    finally:
        L.mx_debug_set(72, old)


@pytest.mark.parametrize("add", [False, True])
def test_assembly_huge_rows(selfcomm, oracle_mod, add):
    """Rows beyond the LDS sort (> 2048 entries): chunk sorts + merge passes,
    with duplicates, negative ids, zeros and rows of exactly 2048 / 2049."""
    from mxsolve.core import DMat
    rng = np.random.default_rng(11 + add)
    M, N = 64, 50000
    lens = rng.integers(0, 30, M)
    lens[[3, 9, 17, 40, 63]] = [2048, 2049, 70001, 9000, 4096]
    ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nnz = int(ip[-1])
    cols = rng.integers(-3, N, nnz).astype(np.int64)
    s40 = slice(ip[40], ip[41])
    cols[s40] = rng.integers(-1, 700, lens[40])      # many duplicates in one huge row
    vals = rng.standard_normal(nnz)
    vals[rng.random(nnz) < 0.05] = 0.0
    A = DMat.from_csr(selfcomm, M, N, ip, cols, vals, add=add)
    O = oracle_mod.OracleMat.from_csr(M, N, ip, cols, vals, P=1, add=add)
    assert_csr_equal(A.csr(), O.csr())


def test_assembly_coo(selfcomm, oracle_mod):
    from mxsolve.core import DMat
    rng = np.random.default_rng(3)
    M = N = 500
    n = 6000
    rows = rng.integers(-1, M, n)
    cols = rng.integers(-1, N, n)
    vals = rng.standard_normal(n)
    for add in (False, True):
        A = DMat.from_coo(selfcomm, M, N, rows, cols, vals, add=add)
        O = oracle_mod.OracleMat.from_coo(M, N, np.array([0, n]), rows, cols, vals, P=1, add=add)
        assert_csr_equal(A.csr(), O.csr())


def test_assembly_errors(selfcomm):
    from mxsolve._lib import MxError
    from mxsolve.core import DMat
    with pytest.raises(MxError) as e:
        DMat.from_csr(selfcomm, 3, 3, np.array([1, 2, 3, 4]), np.array([0, 1, 2]), np.ones(3))
    assert e.value.code == 1
    with pytest.raises(MxError) as e:
        DMat.from_csr(selfcomm, 3, 3, np.array([0, 1, 2, 3]), np.array([0, 1, 7]), np.ones(3))
    assert e.value.code == 2


@pytest.mark.parametrize("kind,n", [("poisson2d", 37), ("poisson3d", 19), ("poisson3d27", 11), ("convdiff3d", 13)])
def test_stencil_generator(selfcomm, oracle_mod, kind, n):
    from mxsolve.core import DMat
    A = DMat.stencil(selfcomm, kind, n)
    assert_csr_equal(A.csr(), oracle_mod.stencil(kind, n))


@pytest.mark.parametrize("kind,n", [("poisson3d", 24), ("poisson3d27", 9), ("convdiff3d", 10)])
def test_spmv_bitexact(selfcomm, oracle_mod, kind, n):
    from mxsolve.core import DMat
    ip, c, v = oracle_mod.stencil(kind, n)
    M = ip.size - 1
    A = DMat.from_csr(selfcomm, M, M, ip, c, v)
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    x = np.random.default_rng(1).standard_normal(M)
    y = torch.zeros(M, dtype=torch.float64, device="cuda")
    A.mult(to_dev(x), y)
    assert np.array_equal(y.cpu().numpy().view(np.uint64), O.mult(x).view(np.uint64))


def test_spmv_bitexact_random(selfcomm, oracle_mod, golden):
    from mxsolve.core import DMat
    A = DMat.from_csr(selfcomm, 100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"])
    O = oracle_mod.OracleMat.from_csr(100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"])
    x = golden["sys_X"]
    y = torch.zeros(100, dtype=torch.float64, device="cuda")
    A.mult(to_dev(x), y)
    assert np.array_equal(y.cpu().numpy(), O.mult(x))


def rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("kind,n,ksp", [("poisson3d", 24, "cg"), ("poisson2d", 64, "cg"),
                                       ("poisson3d27", 12, "cg"), ("convdiff3d", 12, "gmres"),
                                       ("poisson3d", 12, "gmres"),
                                       # odd row counts: the chunk MDot's partial chunk and last row
                                       ("convdiff3d", 13, "gmres"), ("convdiff3d", 29, "gmres")])
def test_ksp_parity(selfcomm, oracle_mod, kind, n, ksp):
    from mxsolve.core import DMat, rhs_hash
    ip, c, v = oracle_mod.stencil(kind, n)
    M = ip.size - 1
    A = DMat.stencil(selfcomm, kind, n)
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    b = torch.zeros(M, dtype=torch.float64, device="cuda")
    rhs_hash(selfcomm, 0, b)
    bh = b.cpu().numpy()
    assert np.array_equal(bh, oracle_mod.rhs_hash(0, M))
    x = torch.zeros(M, dtype=torch.float64, device="cuda")
    r = A.solve(b, x, ksp=ksp, history=True)
    o = O.solve(bh, ksp=ksp, history=True)
    assert r["reason"] == o["reason"] and r["reason"] > 0
    assert r["its"] == o["its"]
    assert rel(x.cpu().numpy(), o["x"]) <= REL_TOL
    assert np.allclose(r["history"], o["history"], rtol=1e-8)


@pytest.mark.parametrize("norm", ["unpreconditioned", "natural", "none"])
def test_cg_norm_types(selfcomm, oracle_mod, norm):
    from mxsolve.core import DMat, rhs_hash
    n = 16
    ip, c, v = oracle_mod.stencil("poisson3d", n)
    M = ip.size - 1
    A = DMat.stencil(selfcomm, "poisson3d", n)
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    b = torch.zeros(M, dtype=torch.float64, device="cuda")
    rhs_hash(selfcomm, 0, b)
    x = torch.zeros(M, dtype=torch.float64, device="cuda")
    kw = dict(max_it=40) if norm == "none" else {}
    r = A.solve(b, x, ksp="cg", norm=norm, **kw)
    o = O.solve(b.cpu().numpy(), ksp="cg", norm=norm, **kw)
    assert (r["its"], r["reason"]) == (o["its"], o["reason"])
    assert rel(x.cpu().numpy(), o["x"]) <= REL_TOL


def test_cg_nonzero_guess_and_maxit(selfcomm, oracle_mod):
    from mxsolve.core import DMat, rhs_hash
    n = 16
    ip, c, v = oracle_mod.stencil("poisson3d", n)
    M = ip.size - 1
    A = DMat.stencil(selfcomm, "poisson3d", n)
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    b = torch.zeros(M, dtype=torch.float64, device="cuda")
    rhs_hash(selfcomm, 0, b)
    x0 = np.sin(np.arange(M))
    x = to_dev(x0)
    r = A.solve(b, x, ksp="cg", guess_nonzero=True)
    o = O.solve(b.cpu().numpy(), x0=x0, ksp="cg")
    assert (r["its"], r["reason"]) == (o["its"], o["reason"])
    assert rel(x.cpu().numpy(), o["x"]) <= REL_TOL
    x = torch.zeros(M, dtype=torch.float64, device="cuda")
    r = A.solve(b, x, ksp="cg", max_it=7)
    o = O.solve(b.cpu().numpy(), ksp="cg", max_it=7)
    assert (r["its"], r["reason"]) == (o["its"], o["reason"]) == (7, -3)
    assert rel(x.cpu().numpy(), o["x"]) <= REL_TOL


def test_cg_zero_rhs(selfcomm):
    from mxsolve.core import DMat
    A = DMat.stencil(selfcomm, "poisson3d", 8)
    b = torch.zeros(512, dtype=torch.float64, device="cuda")
    x = torch.ones(512, dtype=torch.float64, device="cuda")
    r = A.solve(b, x, ksp="cg")
    assert (r["its"], r["reason"]) == (0, 3)
    assert float(x.abs().max()) == 0.0


def test_gmres_reference_system(selfcomm, oracle_mod, golden):
    """test.py's system with -ksp_type gmres -ksp_gmres_restart 100 -pc_type jacobi."""
    from mxsolve.core import DMat
    A = DMat.from_csr(selfcomm, 100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"])
    O = oracle_mod.OracleMat.from_csr(100, 100, golden["sys_indptr"], golden["sys_indices"], golden["sys_data"])
    b = to_dev(golden["sys_B"])
    x = torch.zeros(100, dtype=torch.float64, device="cuda")
    r = A.solve(b, x, ksp="gmres", restart=100, max_it=1000)
    o = O.solve(golden["sys_B"], ksp="gmres", restart=100, max_it=1000)
    assert (r["its"], r["reason"]) == (o["its"], o["reason"])
    assert rel(x.cpu().numpy(), o["x"]) <= 1e-8
    assert np.allclose(x.cpu().numpy(), golden["sys_X"])       # test.py:149's check



@pytest.mark.parametrize("nv", [1, 2, 3, 4, 5, 7, 8, 11, 13, 30])
def test_vec_maxpy_mdot(selfcomm, oracle_mod, nv):
    """mx_vec_maxpy: bit-exact with VecMAXPY_Seq's grouping (first nv % 4, then
    groups of four) for every remainder and pass split; mx_vec_mdot: VecMDot
    within rounding of sequential sums (PETSc leaves the dot order to BLAS)."""
    from mxsolve.core import vmaxpy, vmdot
    rng = np.random.default_rng(nv)
    n = 100_003
    xs_h = [rng.standard_normal(n) for _ in range(nv)]
    y_h = rng.standard_normal(n)
    a = rng.standard_normal(nv)
    xs = [torch.from_numpy(v).cuda() for v in xs_h]
    y = torch.from_numpy(y_h).cuda()
    vmaxpy(selfcomm, y, a, xs)
    got = y.cpu().numpy()
    assert np.array_equal(got.view(np.uint64), oracle_mod.vec_maxpy(y_h, a, xs_h).view(np.uint64))
    d = vmdot(selfcomm, y, xs)
    e = oracle_mod.vec_mdot(got, xs_h)
    assert np.allclose(d, e, rtol=1e-12, atol=1e-9)


def test_ksp_destroy_then_solve(selfcomm, oracle_mod):
    """mx_ksp_destroy (KSPReset) releases the operator's solver state; the next
    solve sets it up again and gives the same bits."""
    from mxsolve.core import DMat, rhs_hash
    A = DMat.stencil(selfcomm, "poisson3d", 16)
    m = A.info()["m"]
    b = selfcomm.empty(m)
    rhs_hash(selfcomm, 0, b)
    x1, x2 = selfcomm.zeros(m), selfcomm.zeros(m)
    r1 = A.solve(b, x1, ksp="cg", pc="jacobi")
    A.ksp_reset()
    A.ksp_reset()                      # idempotent
    r2 = A.solve(b, x2, ksp="cg", pc="jacobi")
    assert r1["its"] == r2["its"] and torch.equal(x1, x2)
    A.destroy()


def test_destroy_current_comm_then_torch(selfcomm):
    """A communicator whose stream is torch's current stream is destroyed,
    then torch allocates and computes at once -- no fixture in between (the
    autouse _selfcomm_stream fixture would re-activate the session stream and
    hide a regression of DeviceComm.destroy's stream hand-back, round 4's
    `HIP error: invalid argument`)."""
    from mxsolve.core import DeviceComm, DMat, rhs_hash
    c = DeviceComm.self_comm(0)
    sp = c.stream_ptr
    assert torch.cuda.current_stream(0).cuda_stream == sp          # creation made it current
    A = DMat.stencil(c, "poisson3d", 16)
    b = c.empty(A.info()["m"])
    rhs_hash(c, 0, b)
    x = c.zeros(A.info()["m"])
    r = A.solve(b, x, ksp="cg")
    assert r["reason"] == 2
    A.destroy()
    c.destroy()
    assert torch.cuda.current_stream(0).cuda_stream != sp
    v = torch.arange(1 << 20, dtype=torch.float64, device="cuda:0")
    w = torch.empty_like(v).copy_(v).mul_(2.0)
    s = float(w.sum())
    torch.cuda.synchronize()
    assert s == float((1 << 20) * ((1 << 20) - 1))


@pytest.mark.parametrize("case", ["dup-insert", "dup-add", "coo-add", "stencil27", "ref"])
def test_assembly_fused_vs_separate(selfcomm, golden, case):
    """Knob 72: the fused canonicalise+split passes (rows <= 64 entries, the
    default) give the separate passes' arrays bit for bit -- CSR, A_d / A_o
    split, diagonal."""
    from mxsolve import _lib
    from mxsolve.core import DMat
    L = _lib.load()
    rng = np.random.default_rng(21)

    def build():
        if case.startswith("dup"):
            M, N = 301, 400
            lens = rng.integers(0, 65, M)
            ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
            nnz = int(ip[-1])
            cols = rng.integers(-2, 90, nnz).astype(np.int64)
            vals = rng.standard_normal(nnz)
            vals[rng.random(nnz) < 0.05] = 0.0
            return lambda: DMat.from_csr(selfcomm, M, N, ip, cols, vals, add=case.endswith("add"))
        if case == "coo-add":
            n = 9000
            r, c, v = rng.integers(-1, 700, n), rng.integers(-1, 700, n), rng.standard_normal(n)
            return lambda: DMat.from_coo(selfcomm, 700, 700, r, c, v, add=True)
        if case == "stencil27":
            return lambda: DMat.stencil(selfcomm, "poisson3d27", 24, 20, 9)
        return lambda: DMat.from_csr(selfcomm, 100, 100, golden["sys_indptr"], golden["sys_indices"],
                                     golden["sys_data"])

    make = build()
    outs = []
    for knob in (1, 0):
        old = L.mx_debug_set(72, knob)
        try:
            A = make()
            d = torch.zeros(A.info()["m"], dtype=torch.float64, device="cuda")
            A.diagonal(d)
            outs.append((A.csr(), A.split(), d.cpu().numpy()))
            A.destroy()
        finally:
            L.mx_debug_set(72, old)
    (c1, s1, d1), (c0, s0, d0) = outs
    for a, b in zip(c1, c0):
        assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    for k in s1:
        assert np.array_equal(np.asarray(s1[k]).view(np.uint8), np.asarray(s0[k]).view(np.uint8)), k
    assert np.array_equal(d1.view(np.uint64), d0.view(np.uint64))


@pytest.mark.parametrize("itype", [np.int32, np.int64])
def test_host_csr_pinned_pieces(selfcomm, oracle_mod, itype):
    """createAIJ(csr=...) from host arrays with one over the registration
    threshold (mx_abi.hip h2d_pinned: 128 MiB; its whole interior pages
    page-locked in chunks ramping from 4 MiB), every array a view that starts
    and ends inside a page, so the partial first and last pages take the plain
    copy; the row pointer and (int32) columns stay under the threshold.  The
    same CSR as the oracle, byte for byte."""
    from mxsolve.core import DMat
    rng = np.random.default_rng(17 + (itype == np.int32))
    M = N = 2_500_000
    lens = rng.integers(5, 10, M)
    ip = np.concatenate([[0], np.cumsum(lens)]).astype(itype)
    nnz = int(ip[-1])
    cols = rng.integers(0, N, nnz).astype(itype)
    vals = rng.standard_normal(nnz)

    def view(a, off):                        # a copy of a, `off` elements into a larger buffer
        buf = np.empty(a.size + off + 5, a.dtype)
        v = buf[off:off + a.size]
        v[:] = a
        return v
    ipv, cv, vv = view(ip, 3), view(cols, 5), view(vals, 1)
    assert vv.nbytes > (128 << 20)
    assert vv.ctypes.data % 4096 and (vv.ctypes.data + vv.nbytes) % 4096
    A = DMat.from_csr(selfcomm, M, N, ipv, cv, vv)
    O = oracle_mod.OracleMat.from_csr(M, N, ip.astype(np.int64), cols.astype(np.int64), vals, P=1)
    assert_csr_equal(A.csr(), O.csr())
    A.destroy()
