"""Generate the golden input fixtures from the reference's own data generators.

Run in the build container (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden.py

The reference scripts cannot be imported as modules here (``import test``
fails with ``ModuleNotFoundError: petsc4py`` -- an ordinary error, not a
permission denial), so this script parses the two source
files with ``ast`` and executes only the pure numpy/scipy generator
functions:

* ``create_system(size, seed, density)``  -- /root/reference/test.py:12-17
* ``create(nsize)``                        -- /root/reference/test2.py:6-18

and then replays the driver's row-block split (test.py:68-91, test2.py:33-50)
on the generated CSR.  The outputs are committed as ``.npz`` data (inputs and
expected outputs only; no reference source text is stored) because
``scipy.sparse.random``'s sampling depends on the numpy/scipy versions
(numpy 2.2.6 / scipy 1.15.3 here).
"""
from __future__ import annotations

import ast
import hashlib
import json
import os
import sys

import numpy as np
import scipy
import scipy.sparse

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _load_function(path: str, name: str, env: dict):
    """Compile and exec one top-level function definition from a source file."""
    with open(path, "r") as f:
        tree = ast.parse(f.read(), filename=path)
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name == name:
            mod = ast.Module(body=[node], type_ignores=[])
            code = compile(mod, filename=path, mode="exec")
            exec(code, env)
            return env[name]
    raise KeyError(f"{name} not found in {path}")


def split_rows(nrows: int, nprocs: int):
    """Driver's divmod split (test.py:68-74) == PetscSplitOwnership."""
    q, r = divmod(nrows, nprocs)
    count = np.array([q + 1 if i < r else q for i in range(nprocs)], dtype=np.int64)
    displ = np.concatenate([[0], np.cumsum(count)[:-1]]).astype(np.int64)
    return count, displ


def sha12(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:12]


def main():
    env = {"np": np, "random": scipy.sparse.random, "csr_matrix": scipy.sparse.csr_matrix}
    create_system = _load_function(os.path.join(REF, "test.py"), "create_system", env)
    create = _load_function(os.path.join(REF, "test2.py"), "create", env)

    A, X, B = create_system(size=100, seed=42, density=0.1)      # test.py:61-62
    A = A.tocsr()
    T = create(100)                                                # test2.py:27-28
    T = T.tocsr()

    out = {
        "sys_indptr": A.indptr.astype(np.int32), "sys_indices": A.indices.astype(np.int32),
        "sys_data": A.data.astype(np.float64), "sys_X": X.astype(np.float64),
        "sys_B": B.astype(np.float64),
        "tri_indptr": T.indptr.astype(np.int32), "tri_indices": T.indices.astype(np.int32),
        "tri_data": T.data.astype(np.float64),
    }
    # expected eigenvalues of the test2 matrix (dense, symmetric)
    ev = np.linalg.eigvalsh(T.toarray())
    out["tri_eigs"] = ev.astype(np.float64)
    # per-rank slices, exactly as the driver builds them (test.py:84-91)
    meta = {"numpy": np.__version__, "scipy": scipy.__version__, "splits": {}}
    for P in (1, 2, 3, 4, 8):
        count, displ = split_rows(100, P)
        meta["splits"][P] = {"count": count.tolist(), "displ": displ.tolist()}
    meta["sha12"] = {k: sha12(v) for k, v in out.items()}
    meta["sys_nnz"] = int(A.nnz)
    meta["sys_has_sorted_indices"] = bool(A.has_sorted_indices)
    meta["sys_zero_diagonals"] = int(np.sum(A.diagonal() == 0))
    meta["tri_nnz"] = int(T.nnz)
    meta["tri_lambda_max"] = float(ev[-1])
    np.savez(os.path.join(HERE, "reference_systems.npz"), **out)
    with open(os.path.join(HERE, "reference_systems.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta["sha12"], indent=1))


if __name__ == "__main__":
    sys.exit(main())
