"""Several PROCESSES on one GPU: the node-local shared-memory transport
(mx_comm_create_shm) that the PETSc shim picks when ranks share GPUs, e.g.
`mpiexec -n 2 python test.py` on a one-GPU machine.

These are the only GPU tests where the distributed path crosses process
boundaries (the in-process LocalComm covers the same kernels and halo plans
at P = 2..8; RCCL refuses two ranks on one device).  The reference's own
call sequences run through examples/ with P = 2 and 4 ranks, and distributed
CG / GMRES solves are checked against the oracle."""
import json
import os
import secrets
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def launch(P, argv, timeout=150):
    port = str(20000 + secrets.randbelow(20000))
    procs = []
    for r in range(P):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(P), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(P),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, *argv], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, cwd=ROOT))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    return [o for o, _ in outs]


@pytest.mark.parametrize("P", [2, 4])
def test_linear_solve_driver_ranks_share_gpu(P):
    """test.py as shipped (preonly + lu) with P ranks on one GPU prints True."""
    outs = launch(P, [os.path.join("examples", "linear_solve_driver.py")])
    assert outs[0].strip().splitlines()[-1] == "True"


def test_linear_solve_driver_gmres_two_ranks():
    """test.py with the Krylov options override (test.py:46), 2 processes."""
    outs = launch(2, [os.path.join("examples", "linear_solve_driver.py"), "-ksp_type", "gmres",
                      "-ksp_gmres_restart", "100", "-pc_type", "jacobi", "-ksp_rtol", "1e-12",
                      "-ksp_converged_reason"])
    lines = outs[0].strip().splitlines()
    assert lines[-1] == "True"
    assert any("CONVERGED_RTOL" in ln for ln in lines)


def test_eigen_driver_two_ranks():
    """test2.py's call sequence (SLEPc EPS HEP) with 2 processes on one GPU."""
    outs = launch(2, [os.path.join("examples", "eigen_driver.py")])
    vals = [float(ln.split()[-1]) for ln in outs[0].splitlines() if ln.startswith("Eigenvalue")]
    assert vals and abs(vals[0] - 558.4042205474284) <= 1e-8 * 558.4


@pytest.mark.parametrize("P,kind,n,ksp", [(2, "poisson3d", 16, "cg"), (3, "poisson3d27", 11, "cg"),
                                         (2, "convdiff3d", 12, "gmres")])
def test_shm_distributed_solve(P, kind, n, ksp):
    """Assembly rows bit-exact, iteration count and reason equal, x within
    1e-10 of the oracle, across processes (1 KiB staging slots: the halo
    and setup exchanges run in several rounds)."""
    name = f"/mxsolve_test_{os.getpid()}_{secrets.token_hex(4)}"
    outs = launch(P, [os.path.join("tests", "_shm_worker.py"), kind, str(n), ksp, name])
    res = json.loads(outs[0].strip().splitlines()[-1])
    assert res["rows_ok"]
    assert (res["its"], res["reason"]) == (res["oracle_its"], res["oracle_reason"]), res
    assert res["rel"] <= 1e-10, res


def test_shm_barrier_then_collectives_skewed():
    """barrier() followed at once by all-reduces / halo exchanges, ranks
    skewed: no false 'ranks entered different collectives' (tags are kept
    per barrier generation), results exact."""
    name = f"/mxsolve_test_{os.getpid()}_{secrets.token_hex(4)}"
    outs = launch(3, [os.path.join("tests", "_shm_stress_worker.py"), "barrier", name], timeout=200)
    for o in outs:
        res = json.loads(o.strip().splitlines()[-1])
        assert res["total"] == res["expect"], res


def test_lu_singular_two_ranks_all_raise():
    """preonly + LU on a singular matrix with 2 processes: rank 0's factorisation
    error reaches every rank as PETSc.Error (no rank left waiting in bcast)."""
    outs = launch(2, [os.path.join("tests", "_shm_stress_worker.py"), "lu_singular", "-"], timeout=120)
    for o in outs:
        res = json.loads(o.strip().splitlines()[-1])
        assert res["raised"], res
