"""mpi4py alias backed by mxsolve.MPI (put mpi-petsc4py-example_amd/compat on
PYTHONPATH to run the reference scripts against the MI355X path unchanged)."""
import os as _os
import sys as _sys

_pkg = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _pkg not in _sys.path:
    _sys.path.insert(0, _pkg)

from mxsolve import MPI  # noqa: E402

_sys.modules[__name__ + ".MPI"] = MPI
