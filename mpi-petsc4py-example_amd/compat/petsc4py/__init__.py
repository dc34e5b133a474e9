"""petsc4py alias backed by mxsolve.PETSc (put mpi-petsc4py-example_amd/compat on
PYTHONPATH to run the reference scripts against the MI355X path unchanged)."""
import os as _os
import sys as _sys

_pkg = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _pkg not in _sys.path:
    _sys.path.insert(0, _pkg)

from mxsolve import PETSc  # noqa: E402

_sys.modules[__name__ + ".PETSc"] = PETSc


def init(args=None, arch=None, comm=None):
    """petsc4py.init(sys.argv) (test.py:5): load argv into the options database."""
    PETSc.init(args, comm)


def get_config():
    return {"PETSC_DIR": _pkg, "PETSC_ARCH": "mi355x-gfx950"}
