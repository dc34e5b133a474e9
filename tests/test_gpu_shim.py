"""The petsc4py/mpi4py/slepc4py-compatible API on the GPU: the reference's call
sequences (test.py, test2.py, petsc_funcs.py) through our from-scratch drivers."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMPAT = os.path.join(ROOT, "mpi-petsc4py-example_amd", "compat")


def run_driver(script, *args, timeout=300):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "examples", script), *args],
                         capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    return out.stdout


def test_linear_solve_driver_lu():
    """test.py as shipped: preonly + lu (mumps) -> prints True (test.py:149)."""
    assert run_driver("linear_solve_driver.py").strip().splitlines()[-1] == "True"


def test_linear_solve_driver_gmres_options():
    """test.py with -ksp_type gmres -ksp_gmres_restart 100 -pc_type jacobi (options override, test.py:46)."""
    out = run_driver("linear_solve_driver.py", "-ksp_type", "gmres", "-ksp_gmres_restart", "100",
                     "-pc_type", "jacobi", "-ksp_converged_reason", "-ksp_rtol", "1e-12")
    lines = out.strip().splitlines()
    assert lines[-1] == "True"
    assert any("Linear solve converged due to CONVERGED_RTOL" in ln for ln in lines)


def test_eigen_driver(golden):
    out = run_driver("eigen_driver.py")
    vals = [float(ln.split()[-1]) for ln in out.splitlines() if ln.startswith("Eigenvalue")]
    assert len(vals) >= 1
    assert abs(vals[0] - 558.4042205474284) <= 1e-8 * 558.4
    ev = golden["tri_eigs"]
    top = ev[np.argsort(-np.abs(ev))][: len(vals)]
    assert np.allclose(vals, top, rtol=1e-8)


@pytest.fixture(scope="module")
def PETSc():
    sys.path.insert(0, COMPAT)
    from mxsolve import PETSc as P
    return P


def test_create_petsc_mat_roundtrip(PETSc, golden):
    from mxsolve import petsc_funcs
    from mxsolve import MPI
    A = petsc_funcs.createPETScMat(MPI.COMM_WORLD, (100, 100),
                                   (golden["sys_indptr"], golden["sys_indices"], golden["sys_data"]))
    ip, cj, vv = A.getValuesCSR()
    assert np.array_equal(ip, golden["sys_indptr"]) and np.array_equal(cj, golden["sys_indices"])
    assert np.array_equal(vv, golden["sys_data"])
    assert A.getSize() == (100, 100) and A.getOwnershipRange() == (0, 100) and A.getType() == "seqaij"
    with pytest.raises(ValueError):
        PETSc.Mat().createAIJ(size=(100, 100), csr=(golden["sys_indptr"][:-1], golden["sys_indices"], golden["sys_data"]))
    with pytest.raises(ValueError):
        PETSc.Mat().createAIJ(size=(100, 100), csr=(golden["sys_indptr"], golden["sys_indices"][:-1], golden["sys_data"]))
    bad = golden["sys_indices"].copy()
    bad[5] = 100
    with pytest.raises(PETSc.Error):
        PETSc.Mat().createAIJ(size=(100, 100), csr=(golden["sys_indptr"], bad, golden["sys_data"]))


def test_setvalues_assembly(PETSc, oracle_mod):
    rng = np.random.default_rng(11)
    n = 60
    A = PETSc.Mat().createAIJ(size=(n, n), nnz=8)
    rows, cols, vals = [], [], []
    for _ in range(300):
        i, j = rng.integers(0, n, 2)
        v = float(rng.integers(-4, 5))
        A.setValue(int(i), int(j), v, addv=PETSc.InsertMode.ADD_VALUES)
        rows.append(i); cols.append(j); vals.append(v)
    A.assemble()
    O = oracle_mod.OracleMat.from_coo(n, n, np.array([0, len(rows)]), np.array(rows), np.array(cols), np.array(vals), add=True)
    ip, cj, vv = A.getValuesCSR()
    oip, ocj, ovv = O.csr()
    assert np.array_equal(ip, oip) and np.array_equal(cj, ocj) and np.array_equal(vv, ovv)


def test_vec_ops(PETSc):
    v = PETSc.Vec().createMPI(1000)
    a = np.sin(np.arange(1000.0))
    v.setArray(a)
    w = v.duplicate()
    w.setArray(np.cos(np.arange(1000.0)))
    assert abs(v.dot(w) - a @ np.cos(np.arange(1000.0))) < 1e-12
    assert abs(v.norm() - np.linalg.norm(a)) < 1e-12
    w.axpy(2.0, v)
    assert np.allclose(w.array, 2.0 * a + np.cos(np.arange(1000.0)), rtol=1e-15, atol=1e-15)
    z = v.duplicate()
    z.pointwiseMult(v, v)
    assert np.array_equal(z.array, a * a)


def test_ksp_cg_options(PETSc, oracle_mod):
    PETSc.Options().setValue("ksp_type", "cg")
    PETSc.Options().setValue("pc_type", "jacobi")
    try:
        ip, c, v = oracle_mod.stencil("poisson3d", 16)
        M = ip.size - 1
        A = PETSc.Mat().createAIJ(size=(M, M), csr=(ip, c, v))
        x, b = A.getVecs()
        b.setArray(oracle_mod.rhs_hash(0, M))
        ksp = PETSc.KSP().create()
        ksp.setType("gmres")           # overridden by the options database
        ksp.setOperators(A)
        ksp.setFromOptions()
        ksp.solve(b, x)
        o = oracle_mod.OracleMat.from_csr(M, M, ip, c, v).solve(oracle_mod.rhs_hash(0, M), ksp="cg")
        assert ksp.getType() == "cg"
        assert ksp.getIterationNumber() == o["its"] and ksp.getConvergedReason() == o["reason"]
        assert np.linalg.norm(x.array - o["x"]) / np.linalg.norm(o["x"]) <= 1e-10
        assert abs(ksp.getResidualNorm() - o["rnorm"]) <= 1e-8 * o["rnorm"]
    finally:
        PETSc.Options().delValue("ksp_type")
        PETSc.Options().delValue("pc_type")


def test_ksp_not_converged_does_not_raise(PETSc, oracle_mod):
    ip, c, v = oracle_mod.stencil("poisson3d", 12)
    M = ip.size - 1
    A = PETSc.Mat().createAIJ(size=(M, M), csr=(ip, c, v))
    x, b = A.getVecs()
    b.set(1.0)
    ksp = PETSc.KSP().create()
    ksp.setType("cg")
    ksp.getPC().setType("jacobi")
    ksp.setTolerances(rtol=1e-12, max_it=5)
    ksp.setOperators(A)
    ksp.solve(b, x)
    assert ksp.getConvergedReason() == PETSc.KSP.ConvergedReason.DIVERGED_ITS
    assert ksp.getIterationNumber() == 5


def test_binary_viewer_roundtrip(PETSc, golden, tmp_path):
    """Mat/Vec view -> load through a binary viewer (F4), values bit-identical."""
    A = PETSc.Mat().createAIJ(size=(100, 100), csr=(golden["sys_indptr"], golden["sys_indices"], golden["sys_data"]))
    x, b = A.getVecs()
    b.setArray(golden["sys_B"])
    fn = str(tmp_path / "a.bin")
    with PETSc.Viewer().createBinary(fn, "w") as vw:
        A.view(vw)
        b.view(vw)
    with PETSc.Viewer().createBinary(fn, "r") as vr:
        A2 = PETSc.Mat().load(vr)
        b2 = PETSc.Vec().load(vr)
    for u, v in zip(A2.getValuesCSR(), A.getValuesCSR()):
        assert np.array_equal(u, v)
    assert np.array_equal(b2.array, golden["sys_B"])


def test_ksp_destroy_keeps_shared_operator_state(PETSc):
    """Two KSPs on one Mat: destroying one leaves the other's solver state on
    the operator (PETSc's KSPDestroy leaves the Mat alone) -- its next solve
    gives the same bits; the last user's reset releases the state and the Mat
    still multiplies."""
    from mxsolve.core import dispatch_counts
    n = 32
    A = PETSc.Mat().createAIJ(size=(n ** 3, n ** 3), csr=_poisson3d_csr(n))
    A.assemble()
    x, b = A.getVecs()
    b.setArray(np.linspace(0.0, 1.0, n ** 3))
    k1, k2 = PETSc.KSP().create(), PETSc.KSP().create()
    for k in (k1, k2):
        k.setType("cg")
        k.getPC().setType("jacobi")
        k.setOperators(A)
    k1.solve(b, x)
    x1 = x.array.copy()
    x.set(0.0)
    k2.solve(b, x)
    assert np.array_equal(x.array.view(np.uint64), x1.view(np.uint64))
    assert A._ksp_users == 2
    k1.destroy()
    assert A._ksp_users == 1 and A.getDeviceHandle().h
    x.set(0.0)
    k2.solve(b, x)
    assert np.array_equal(x.array.view(np.uint64), x1.view(np.uint64))
    k2.destroy()
    assert A._ksp_users == 0
    y = x.duplicate()
    A.mult(b, y)
    assert np.isfinite(y.array).all()


def _poisson3d_csr(n):
    import itertools
    rows, cols, vals = [], [], []
    ip = [0]
    for k, j, i in itertools.product(range(n), range(n), range(n)):
        r = i + n * j + n * n * k
        for dk, dj, di, v in ((-1, 0, 0, -1.0), (0, -1, 0, -1.0), (0, 0, -1, -1.0), (0, 0, 0, 6.0),
                              (0, 0, 1, -1.0), (0, 1, 0, -1.0), (1, 0, 0, -1.0)):
            kk, jj, ii = k + dk, j + dj, i + di
            if 0 <= kk < n and 0 <= jj < n and 0 <= ii < n:
                cols.append(ii + n * jj + n * n * kk)
                vals.append(v)
        ip.append(len(cols))
    return np.array(ip, np.int32), np.array(cols, np.int32), np.array(vals)


def test_binary_viewer_known_bytes(PETSc, tmp_path):
    """Mat.view / Vec.view through a binary viewer on a matrix assembled on the
    GPU (unsorted input columns: the file holds the assembled, sorted rows)
    write PETSc's documented bytes -- the literal stream of
    tests/test_cpu_shim.py::test_petsc_binary_known_bytes."""
    expected = bytes.fromhex(
        "00127b50" "00000003" "00000003" "00000005" "00000001" "00000002" "00000002"
        "00000000" "00000000" "00000001" "00000001" "00000002"
        "4000000000000000" "bff0000000000000" "4008000000000000" "3fe0000000000000" "c010000000000000"
        "00127b4e" "00000003" "3ff8000000000000" "c000000000000000" "0000000000000000")
    ip = np.array([0, 1, 3, 5], dtype=np.int32)
    cj = np.array([0, 1, 0, 2, 1], dtype=np.int32)
    vv = np.array([2.0, 3.0, -1.0, -4.0, 0.5])
    A = PETSc.Mat().createAIJ(size=(3, 3), csr=(ip, cj, vv))
    A.assemble()
    x, b = A.getVecs()
    b.setArray(np.array([1.5, -2.0, 0.0]))
    fn = tmp_path / "k.bin"
    with PETSc.Viewer().createBinary(str(fn), "w") as vw:
        A.view(vw)
        b.view(vw)
    assert fn.read_bytes() == expected


def test_ascii_view_petsc_format(PETSc, capsys):
    """A.view() / b.view() (petsc_funcs.py:8, commented out in the reference)
    print PETSc's default ASCII format: "row i: (j, v) ..." with "%g" values."""
    ip = np.array([0, 2, 5, 7], dtype=np.int32)
    cj = np.array([0, 1, 0, 1, 2, 1, 2], dtype=np.int32)
    vv = np.array([2.0, -1.0, -1.0, 2.0, -1.0, -1.0, 2.5])
    A = PETSc.Mat().createAIJ(size=(3, 3), csr=(ip, cj, vv))
    A.assemble()
    capsys.readouterr()
    A.view()
    out = capsys.readouterr().out.splitlines()
    assert out == ["Mat Object: 1 MPI process", "  type: seqaij",
                   "row 0: (0, 2.)  (1, -1.) ", "row 1: (0, -1.)  (1, 2.)  (2, -1.) ", "row 2: (1, -1.)  (2, 2.5) "]
    x, b = A.getVecs()
    b.setArray(np.array([1.0, 0.5, 3e-7]))
    b.view()
    out = capsys.readouterr().out.splitlines()
    assert out == ["Vec Object: 1 MPI process", "  type: seq", "1.", "0.5", "3e-07"]


def test_insert_values_explicit_over_existing(PETSc):
    """An explicit INSERT_VALUES replaces existing entries (Vec and Mat re-assembly);
    ADD_VALUES sums into them."""
    from mxsolve import MPI
    v = PETSc.Vec().createMPI(4, comm=MPI.COMM_WORLD)
    v.set(1.0)
    v.setValues([0, 2], [5.0, 7.0], PETSc.InsertMode.INSERT_VALUES)
    v.assemble()
    assert np.array_equal(v.getArray(), [5.0, 1.0, 7.0, 1.0])
    w = PETSc.Vec().createMPI(4, comm=MPI.COMM_WORLD)
    w.set(1.0)
    w.setValues([1], [2.5], PETSc.InsertMode.ADD_VALUES)
    w.assemble()
    assert np.array_equal(w.getArray(), [1.0, 3.5, 1.0, 1.0])

    A = PETSc.Mat().create(comm=MPI.COMM_WORLD)
    A.setSizes((3, 3))
    A.setUp()
    for i in range(3):
        A.setValues([i], [i], [[2.0]], PETSc.InsertMode.INSERT_VALUES)
    A.assemble()
    A.setValues([1], [1], [[9.0]], PETSc.InsertMode.INSERT_VALUES)
    A.setValuesCSR([0, 1, 1, 1], [0], [4.0], PETSc.InsertMode.INSERT_VALUES)
    A.assemble()
    assert np.array_equal(A.getDiagonal().getArray(), [4.0, 9.0, 2.0])
    A.setValues([2], [2], [[1.5]], PETSc.InsertMode.ADD_VALUES)
    A.assemble()
    assert np.array_equal(A.getDiagonal().getArray(), [4.0, 9.0, 3.5])
