"""petsc4py-compatible operator API over libmxsolve.so.

Covers every PETSc call the reference makes:
  petsc_funcs.py:6-7   Mat().createAIJ(comm, size, csr) + assemble()
  test.py:24-30        createAIJ, setUp, assemblyBegin/End, getVecs, Vec.setArray
  test.py:33-50        KSP().create, setType, getPC, PC.setType,
                       PC.setFactorSolverType, setOperators, setFromOptions,
                       setUp, solve
  test.py:145          Vec.array
  test.py:5            petsc4py.init(sys.argv) -> the options database
plus the harness calls the parity/bench drivers need (getValuesCSR,
getOwnershipRange, mult, getDiagonal, getIterationNumber, getConvergedReason,
getResidualNorm, setTolerances, Vec.norm/dot/duplicate/set, MatSetValues).

Semantics kept from petsc4py/PETSc: objects are collective on their
communicator; createAIJ and setArray copy their inputs; bad CSR arguments
raise ValueError; library failures raise PETSc.Error (a RuntimeError with
.ierr); a Krylov solve that does not converge does not raise, it sets a
negative converged reason (unless -ksp_error_if_not_converged).

Device layout: every Vec owns a float64 torch tensor of its local rows in
HBM; every Mat is an mx_mat handle.  Nothing here computes on the CPU: the
matrix, vector and solver operations are libmxsolve.so calls.
"""
from __future__ import annotations

import os
import shlex
import sys
import time

import numpy as np
import torch

from . import MPI as _MPI
from . import _lib, core

# ------------------------------------------------------------------ errors
PETSC_ERR_MEM, PETSC_ERR_SUP, PETSC_ERR_ARG_OUTOFRANGE, PETSC_ERR_LIB, PETSC_ERR_ARG_WRONG = 55, 56, 63, 76, 62
DECIDE = -1
DEFAULT = -2
DETERMINE = -1
UNLIMITED = -3


class Error(RuntimeError):
    """PETSc.Error: carries the PETSc error code in .ierr."""

    def __init__(self, ierr: int = PETSC_ERR_LIB, msg: str = ""):
        self.ierr = ierr
        super().__init__(f"error code {ierr}" + (f"\n{msg}" if msg else ""))


def _raise(e: _lib.MxError):
    if e.code == _lib.MX_ERR_ARG:
        raise ValueError(e.msg) from None
    code = {_lib.MX_ERR_OUTOFRANGE: PETSC_ERR_ARG_OUTOFRANGE, _lib.MX_ERR_MEM: PETSC_ERR_MEM,
            _lib.MX_ERR_UNSUPPORTED: PETSC_ERR_SUP}.get(e.code, PETSC_ERR_LIB)
    raise Error(code, e.msg) from None


def _guard(fn, *a, **k):
    try:
        return fn(*a, **k)
    except _lib.MxError as e:
        _raise(e)


# ------------------------------------------------------------------ options database
_OPTS: dict[str, str | None] = {}


def _parse_argv(argv):
    out, i = {}, 0
    while i < len(argv):
        a = argv[i]
        if isinstance(a, str) and a.startswith("-") and len(a) > 1 and not _is_number(a):
            key = a.lstrip("-")
            if i + 1 < len(argv) and not (str(argv[i + 1]).startswith("-") and not _is_number(str(argv[i + 1]))):
                out[key] = str(argv[i + 1])
                i += 2
                continue
            out[key] = None
        i += 1
    return out


def _is_number(s: str) -> bool:
    try:
        float(s)
        return True
    except ValueError:
        return False


def _init_options(argv=None):
    env = os.environ.get("PETSC_OPTIONS", "")
    if env:
        _OPTS.update(_parse_argv(shlex.split(env)))
    if argv:
        _OPTS.update(_parse_argv(list(argv)[1:]))


_init_options()


class Options:
    """PETSc options database (PetscOptions) with an optional prefix."""

    def __init__(self, prefix: str | None = None):
        self.prefix = prefix or ""

    def _k(self, name: str) -> str:
        return self.prefix + name.lstrip("-")

    def hasName(self, name):
        return self._k(name) in _OPTS

    def setValue(self, name, value):
        _OPTS[self._k(name)] = None if value is None else str(value)

    def delValue(self, name):
        _OPTS.pop(self._k(name), None)

    def getString(self, name, default=None):
        v = _OPTS.get(self._k(name), default)
        return default if v is None else v

    def getInt(self, name, default=None):
        v = _OPTS.get(self._k(name))
        return default if v is None else int(float(v))

    def getReal(self, name, default=None):
        v = _OPTS.get(self._k(name))
        return default if v is None else float(v)

    def getBool(self, name, default=None):
        k = self._k(name)
        if k not in _OPTS:
            return default
        v = _OPTS[k]
        return True if v is None else v.lower() in ("1", "true", "yes", "on")

    def getAll(self):
        return dict(_OPTS)

    def __contains__(self, name):
        return self.hasName(name)

    def __getitem__(self, name):
        return self.getString(name)

    def __setitem__(self, name, value):
        self.setValue(name, value)

    def __delitem__(self, name):
        self.delValue(name)


# ------------------------------------------------------------------ communicators
class Comm:
    """PETSc.Comm wrapping an mpi4py-compatible communicator."""

    def __init__(self, mpi_comm=None):
        self.tompi4py_comm = mpi_comm if mpi_comm is not None else _MPI.COMM_WORLD

    def tompi4py(self):
        return self.tompi4py_comm

    def getRank(self):
        return self.tompi4py_comm.Get_rank()

    def getSize(self):
        return self.tompi4py_comm.Get_size()

    rank = property(getRank)
    size = property(getSize)

    def barrier(self):
        self.tompi4py_comm.Barrier()


COMM_WORLD = Comm(_MPI.COMM_WORLD)
COMM_SELF = Comm(_MPI.COMM_SELF)

_DEVICE_COMMS: dict[int, core.DeviceComm] = {}


def _petsc_g(v) -> str:
    """PETSc's "%g": a value that prints like an integer gets a trailing '.'."""
    t = f"{float(v):g}"
    return t if any(ch in t for ch in ".eEn") else t + "."


def _mpi(comm):
    if comm is None:
        return _MPI.COMM_WORLD
    if isinstance(comm, Comm):
        return comm.tompi4py_comm
    return comm


def _transport(mc) -> str:
    """RCCL when every rank of the node has a GPU of its own; the shared-memory
    transport when ranks share GPUs (RCCL refuses two ranks on one device).
    MXSOLVE_TRANSPORT=rccl|shm overrides.  Decided on rank 0, broadcast."""
    choice = None
    if mc.Get_rank() == 0:
        choice = os.environ.get("MXSOLVE_TRANSPORT", "").lower()
        if choice not in ("rccl", "shm"):
            import torch
            local = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", mc.Get_size())))
            choice = "shm" if local > torch.cuda.device_count() else "rccl"
    return mc.bcast(choice, root=0)


def _device_comm(comm) -> core.DeviceComm:
    """One libmxsolve communicator per MPI communicator: self for one rank,
    RCCL (unique id broadcast over the host control plane) or, when ranks
    share GPUs, the node-local shared-memory transport."""
    mc = _mpi(comm)
    key = id(mc)
    dc = _DEVICE_COMMS.get(key)
    if dc is None:
        if mc.Get_size() == 1:
            dc = _guard(core.DeviceComm.self_comm)
        elif _transport(mc) == "shm":
            import secrets
            name = f"/mxsolve_{os.getpid()}_{secrets.token_hex(6)}" if mc.Get_rank() == 0 else None
            name = mc.bcast(name, root=0)
            dc = _guard(core.DeviceComm.shm, mc.Get_rank(), mc.Get_size(), name)
        else:
            uid = _guard(core.unique_id) if mc.Get_rank() == 0 else None
            uid = mc.bcast(uid, root=0)
            dc = _guard(core.DeviceComm.rccl, mc.Get_rank(), mc.Get_size(), uid)
        _DEVICE_COMMS[key] = dc
    dc.activate()
    return dc


def _sizes(size, comm_size, rank):
    """petsc4py size forms: N | (n, N) | (M, N) | ((m, M), (n, N)) -> (m, M) pairs."""
    def one(s):
        if isinstance(s, (tuple, list)):
            n, N = s
            n = DECIDE if n is None else int(n)
            N = DETERMINE if N is None else int(N)
            if N < 0:
                N = _MPI.COMM_WORLD.allreduce(n) if comm_size > 1 else n
            return n, N
        return DECIDE, int(s)
    if isinstance(size, (tuple, list)) and len(size) == 2 and all(isinstance(s, (tuple, list)) for s in size):
        return one(size[0]), one(size[1])
    if isinstance(size, (tuple, list)) and len(size) == 2:
        return (DECIDE, int(size[0])), (DECIDE, int(size[1]))
    r = one(size)
    return r, r


def _split(N, P, r):
    q, rem = divmod(N, P)
    start = r * q + min(r, rem)
    return start, q + (1 if r < rem else 0)


# ------------------------------------------------------------------ Viewer (binary)
class Viewer:
    """PETSc binary viewer (PetscViewerBinaryOpen): Mat/Vec in PETSc's file format.
    Rank 0 writes the gathered object; every rank reads the file and keeps its rows."""

    class Mode:
        READ, WRITE, APPEND = "r", "w", "a"
        R, W, A = "r", "w", "a"

    class Format:
        DEFAULT, ASCII_INFO = 0, 1

    def __init__(self):
        self._fh = None
        self._mode = None
        self._comm = None
        self._name = None

    def createBinary(self, name, mode="r", comm=None):
        self._comm = Comm(_mpi(comm))
        self._name = str(name)
        self._mode = {"r": "rb", "w": "wb", "a": "ab"}[str(mode)[0].lower()]
        mc = _mpi(comm)
        if self._mode == "rb" or mc.Get_rank() == 0:
            self._fh = open(self._name, self._mode)
        return self

    def destroy(self):
        if self._fh:
            self._fh.close()
            self._fh = None
        return self

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.destroy()


# ------------------------------------------------------------------ Vec
class Vec:
    """Distributed vector; the local rows live in a float64 tensor in HBM."""

    class Type:
        SEQ, MPI, STANDARD, CUDA, HIP = "seq", "mpi", "standard", "cuda", "hip"

    class Option:
        IGNORE_NEGATIVE_INDICES = 1

    def __init__(self):
        self._t = None
        self._dc = None
        self._comm = None
        self._N = 0
        self._rstart = 0

    # -- creation -------------------------------------------------------------
    def _setup(self, comm, n_local, N):
        mc = _mpi(comm)
        P, r = mc.Get_size(), mc.Get_rank()
        if n_local < 0:
            self._rstart, n_local = _split(N, P, r)
        else:
            starts = mc.allgather(n_local) if P > 1 else [n_local]
            self._rstart = int(sum(starts[:r]))
            if sum(starts) != N:
                raise Error(PETSC_ERR_ARG_WRONG, f"Sum of local lengths {sum(starts)} does not equal global length {N}")
        self._comm = comm if isinstance(comm, Comm) else Comm(mc)
        self._dc = _device_comm(mc)
        self._N = int(N)
        self._t = self._dc.zeros(n_local)
        return self

    def create(self, comm=None):
        self._comm = comm if isinstance(comm, Comm) else Comm(_mpi(comm))
        return self

    @staticmethod
    def _vsize(size, mc):
        """Vec sizes: N | (n, N) with None / DECIDE / DETERMINE entries."""
        if isinstance(size, (tuple, list)):
            n, N = size
            n = DECIDE if n is None else int(n)
            N = DETERMINE if N is None else int(N)
            if N < 0:
                N = mc.allreduce(n) if mc.Get_size() > 1 else n
            return n, N
        return DECIDE, int(size)

    def setSizes(self, size, bsize=None):
        mc = _mpi(self._comm)
        n, N = self._vsize(size, mc)
        return self._setup(mc, n, N)

    def setType(self, t):
        return self

    def setUp(self):
        return self

    def setFromOptions(self):
        return self

    def createMPI(self, size, bsize=None, comm=None):
        mc = _mpi(comm)
        n, N = self._vsize(size, mc)
        return self._setup(mc, n, N)

    def createSeq(self, size, bsize=None, comm=None):
        n = size if not isinstance(size, (tuple, list)) else size[0]
        return self._setup(_MPI.COMM_SELF, int(n), int(n))

    def duplicate(self, array=None):
        v = Vec()
        v._comm, v._dc, v._N, v._rstart = self._comm, self._dc, self._N, self._rstart
        self._dc.activate()
        v._t = self._dc.zeros(self._t.numel())
        if array is not None:
            v.setArray(array)
        return v

    def copy(self, result=None):
        if result is None:
            result = self.duplicate()
        self._dc.activate()
        result._t.copy_(self._t)
        return result

    def destroy(self):
        self._t = None
        return self

    # -- sizes --------------------------------------------------------------------
    def getSize(self):
        return self._N

    def getLocalSize(self):
        return int(self._t.numel())

    def getSizes(self):
        return (self.getLocalSize(), self._N)

    def getOwnershipRange(self):
        return (self._rstart, self._rstart + self.getLocalSize())

    def getComm(self):
        return self._comm

    size = property(getSize)
    local_size = property(getLocalSize)
    sizes = property(getSizes)
    owner_range = property(getOwnershipRange)

    # -- data movement -------------------------------------------------------------
    def setArray(self, array):
        """Copies the local values in (test.py:30)."""
        a = np.ascontiguousarray(array, dtype=np.float64).reshape(-1)
        if a.size != self.getLocalSize():
            raise ValueError(f"array size {a.size} and vector local size {self.getLocalSize()} incompatible")
        self._dc.activate()
        self._t.copy_(torch.from_numpy(a))
        return self

    placeArray = setArray

    def getArray(self, readonly=False):
        """Host copy of the local values (a device vector cannot be mapped in place)."""
        self._dc.activate()
        return self._t.cpu().numpy()

    array = property(getArray, setArray)
    array_r = property(getArray)

    def setValues(self, indices, values, addv=None):
        """VecSetValues: owned entries are applied now, the others go to the
        stash and reach their owner at assemblyEnd (negative indices skipped)."""
        gidx = np.atleast_1d(np.asarray(indices, dtype=np.int64))
        val = np.broadcast_to(np.asarray(values, dtype=np.float64), gidx.shape)
        add = _is_add(addv)
        mode = getattr(self, "_vmode", None)
        if mode is not None and mode != add:
            raise Error(PETSC_ERR_ARG_WRONG, "You have already added values; you cannot now insert")
        self._vmode = add
        keep = gidx >= 0
        if np.any(gidx[keep] >= self._N):
            raise Error(PETSC_ERR_ARG_OUTOFRANGE, f"Out of range index value {int(gidx[keep].max())} maximum {self._N}")
        lo, hi = self.getOwnershipRange()
        own = keep & (gidx >= lo) & (gidx < hi)
        off = keep & ~own
        if np.any(off):
            self._vstash = getattr(self, "_vstash", []) + [(gidx[off].copy(), val[off].copy())]
        if np.any(own):
            host = self.getArray()
            if add:
                np.add.at(host, gidx[own] - lo, val[own])
            else:
                host[gidx[own] - lo] = val[own]
            self.setArray(host)

    def setValue(self, index, value, addv=None):
        self.setValues([index], [value], addv)

    def assemblyBegin(self):
        return self

    def assemblyEnd(self):
        """VecAssemblyEnd: deliver the stash (collective).  Entries arrive in
        ascending source-rank order, each rank's in call order."""
        mc = _mpi(self._comm)
        stash = getattr(self, "_vstash", [])
        add = getattr(self, "_vmode", None)
        if mc.Get_size() > 1:
            mine = (np.concatenate([s[0] for s in stash]) if stash else np.zeros(0, np.int64),
                    np.concatenate([s[1] for s in stash]) if stash else np.zeros(0))
            every = mc.allgather((mine, add))
            modes = {m for (_, m) in every if m is not None}
            if len(modes) > 1:
                raise Error(PETSC_ERR_ARG_WRONG, "Some processors inserted values while others added")
            lo, hi = self.getOwnershipRange()
            got = [(i[(i >= lo) & (i < hi)], v[(i >= lo) & (i < hi)]) for (i, v), _ in every]
            if any(g[0].size for g in got):
                host = self.getArray()
                for i, v in got:
                    if modes == {True}:
                        np.add.at(host, i - lo, v)
                    else:
                        host[i - lo] = v
                self.setArray(host)
        self._vstash, self._vmode = [], None
        return self

    def assemble(self):
        self.assemblyBegin()
        return self.assemblyEnd()

    # -- algebra (all through libmxsolve) -------------------------------------------
    def set(self, alpha):
        _guard(core.vset, self._dc, alpha, self._t)

    def zeroEntries(self):
        self.set(0.0)

    def scale(self, alpha):
        _guard(core.vscale, self._dc, alpha, self._t)

    def axpy(self, alpha, x):
        _guard(core.vaxpy, self._dc, alpha, x._t, self._t)

    def aypx(self, alpha, x):
        _guard(core.vaypx, self._dc, alpha, x._t, self._t)

    def pointwiseMult(self, x, y):
        _guard(core.vpmult, self._dc, x._t, y._t, self._t)

    def dot(self, v):
        # VecDot(x, y) = y^H x; real scalars
        return _guard(core.vdot, self._dc, self._t, v._t)

    tDot = dot

    def norm(self, norm_type=None):
        if norm_type not in (None, NormType.NORM_2, NormType.FROBENIUS):
            raise Error(PETSC_ERR_SUP, "only the 2-norm is implemented")
        return _guard(core.vnorm, self._dc, self._t)

    def normalize(self):
        nrm = self.norm()
        if nrm != 0.0:
            self.scale(1.0 / nrm)
        return nrm

    def view(self, viewer=None):
        from . import petsc_io
        arr = self.getArray()
        mc = _mpi(self._comm)
        if isinstance(viewer, Viewer):
            parts = mc.allgather(arr) if mc.Get_size() > 1 else [arr]
            if mc.Get_rank() == 0:
                petsc_io.write_vec(viewer._fh, np.concatenate(parts))
                viewer._fh.flush()
            return
        # VecView_MPI_ASCII default format: values per process, "%g"
        P = mc.Get_size()
        parts = mc.allgather(arr) if P > 1 else [arr]
        if mc.Get_rank() == 0:
            lines = [f"Vec Object: {P} MPI process{'es' if P > 1 else ''}", f"  type: {'mpi' if P > 1 else 'seq'}"]
            for q, a in enumerate(parts):
                if P > 1:
                    lines.append(f"Process [{q}]")
                lines += [_petsc_g(v) for v in a]
            print("\n".join(lines), flush=True)

    def load(self, viewer):
        """VecLoad: the next Vec in a binary viewer, split by PetscSplitOwnership."""
        from . import petsc_io
        vals = petsc_io.read_vec(viewer._fh)
        mc = _mpi(viewer._comm)
        self._setup(mc, -1, vals.size)
        a, b = self.getOwnershipRange()
        self.setArray(vals[a:b])
        return self

    def __len__(self):
        return self.getLocalSize()

    # device tensor for in-framework consumers
    def getDeviceTensor(self):
        return self._t


class NormType:
    NORM_1, NORM_2, FROBENIUS, INFINITY, NORM_1_AND_2 = 0, 1, 2, 3, 4
    N1, N2, NINF = 0, 1, 3


class InsertMode:
    INSERT_VALUES = INSERT = 1
    ADD_VALUES = ADD = 2
    NOT_SET_VALUES = 0


def _is_add(addv) -> bool:
    """petsc4py's InsertMode argument: None/False insert, True adds, an int is
    compared against ADD_VALUES only (INSERT_VALUES == 1 == True must not add)."""
    if addv is None or isinstance(addv, bool):
        return addv is True
    return int(addv) == InsertMode.ADD_VALUES


# ------------------------------------------------------------------ Mat
class Mat:
    """Row-partitioned AIJ matrix (MATSEQAIJ / MATMPIAIJ)."""

    class Type:
        AIJ, SEQAIJ, MPIAIJ, DENSE = "aij", "seqaij", "mpiaij", "dense"

    class Option:
        NEW_NONZERO_ALLOCATION_ERR = 19
        IGNORE_ZERO_ENTRIES = 24

    class AssemblyType:
        FINAL_ASSEMBLY, FLUSH_ASSEMBLY = 0, 1
        FINAL, FLUSH = 0, 1

    def __init__(self):
        self._h = None
        self._comm = None
        self._dc = None
        self._size = None
        self._stash = []       # pending setValues: (rows, cols, vals)
        self._mode = None

    # -- creation ---------------------------------------------------------------------
    def createAIJ(self, size, bsize=None, nnz=None, csr=None, comm=None):
        """Mat().createAIJ(comm=comm, size=shape, csr=(indptr, indices, data))
        (petsc_funcs.py:6, test.py:24): copies the local CSR (global column ids)
        and assembles it on the GPU."""
        mc = _mpi(comm)
        self._comm = Comm(mc)
        (m, M), (n, N) = _sizes(size, mc.Get_size(), mc.Get_rank())
        self._size = (m, M, n, N)
        self._dc = _device_comm(mc)
        if csr is not None:
            if len(csr) == 3:
                ip, cj, vv = csr
            elif len(csr) == 2:
                ip, cj = csr
                vv = np.zeros(len(cj))
            else:
                raise ValueError("csr must be (I, J[, V])")
            self._from_csr(ip, cj, vv)
        return self

    createAIJWithArrays = createAIJ

    def _local_rows(self):
        m, M, _, _ = self._size
        mc = _mpi(self._comm)
        return _split(M, mc.Get_size(), mc.Get_rank())[1] if m < 0 else m

    def _from_csr(self, ip, cj, vv):
        ip = np.ascontiguousarray(ip)
        cj = np.ascontiguousarray(cj)
        vv = np.ascontiguousarray(vv, dtype=np.float64)
        if ip.dtype.kind not in "iu":
            raise TypeError("I must be an integer array")
        m = self._local_rows()
        # petsc4py Mat_AllocAIJ_CSR argument checks
        if ip.size - 1 != m:
            raise ValueError(f"size(I) is {ip.size}, expected {m + 1}")
        if int(ip[0]) != 0:
            raise ValueError(f"I[0] is {int(ip[0])}, expected 0")
        if int(ip[-1]) != cj.size:
            raise ValueError(f"size(J) is {cj.size}, expected {int(ip[-1])}")
        if vv.size != int(ip[-1]):
            raise ValueError(f"size(V) is {vv.size}, expected {int(ip[-1])}")
        m_, M, n_, N = self._size
        self._dc.activate()
        self._h = _guard(core.DMat.from_csr, self._dc, M, N, ip, cj, vv, m_local=m_, n_local=n_)

    def create(self, comm=None):
        self._comm = Comm(_mpi(comm))
        return self

    def setSizes(self, size, bsize=None):
        mc = _mpi(self._comm)
        (m, M), (n, N) = _sizes(size, mc.Get_size(), mc.Get_rank())
        self._size = (m, M, n, N)
        self._dc = _device_comm(mc)
        return self

    def setType(self, t):
        return self

    def setFromOptions(self):
        return self

    def setPreallocationNNZ(self, nnz):
        return self

    def setPreallocationCSR(self, csr):
        ip, cj, vv = csr if len(csr) == 3 else (*csr, np.zeros(len(csr[1])))
        self._from_csr(ip, cj, vv)
        return self

    def setOption(self, option, flag):
        return self

    def setUp(self):
        return self

    # -- MatSetValues-style assembly -----------------------------------------------------
    def setValues(self, rows, cols, values, addv=None):
        rows = np.atleast_1d(np.asarray(rows, dtype=np.int64))
        cols = np.atleast_1d(np.asarray(cols, dtype=np.int64))
        vals = np.asarray(values, dtype=np.float64).reshape(rows.size, cols.size)
        mode = InsertMode.ADD_VALUES if _is_add(addv) else InsertMode.INSERT_VALUES
        if self._mode is not None and mode != self._mode:
            raise Error(PETSC_ERR_ARG_WRONG, "You cannot mix add values and insert values")
        self._mode = mode
        R = np.repeat(rows, cols.size)
        Cc = np.tile(cols, rows.size)
        self._stash.append((R, Cc, vals.reshape(-1)))

    def setValue(self, row, col, value, addv=None):
        self.setValues([row], [col], [[value]], addv)

    def setValuesCSR(self, I, J, V, addv=None):
        I = np.asarray(I, dtype=np.int64)
        rstart = self.getOwnershipRange()[0] if self._h else _split(self._size[1], self._comm.size, self._comm.rank)[0]
        rows = np.repeat(np.arange(I.size - 1, dtype=np.int64) + rstart, np.diff(I))
        mode = InsertMode.ADD_VALUES if _is_add(addv) else InsertMode.INSERT_VALUES
        self._mode = self._mode or mode
        self._stash.append((rows, np.asarray(J, dtype=np.int64), np.asarray(V, dtype=np.float64)))

    def assemblyBegin(self, assembly=None):
        return self

    def assemblyEnd(self, assembly=None):
        if not self._stash:
            if self._h is None and self._size is not None:
                self._stash.append((np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0)))
            else:
                return self
        rows = np.concatenate([s[0] for s in self._stash])
        cols = np.concatenate([s[1] for s in self._stash])
        vals = np.concatenate([s[2] for s in self._stash])
        add = self._mode == InsertMode.ADD_VALUES
        if self._h is not None:
            # re-assembly: existing entries first, then the new ones in order
            ip, cj, vv = self._h.csr()
            r0 = self.getOwnershipRange()[0]
            er = np.repeat(np.arange(ip.size - 1, dtype=np.int64) + r0, np.diff(ip))
            rows, cols, vals = np.concatenate([er, rows]), np.concatenate([cj, cols]), np.concatenate([vv, vals])
        m_, M, n_, N = self._size
        self._dc.activate()
        self._h = _guard(core.DMat.from_coo, self._dc, M, N, rows, cols, vals, m_local=m_, n_local=n_, add=add)
        self._stash, self._mode = [], None
        return self

    def assemble(self, assembly=None):
        self.assemblyBegin(assembly)
        return self.assemblyEnd(assembly)

    def isAssembled(self):
        return self._h is not None and not self._stash

    # -- queries ---------------------------------------------------------------------------
    def _info(self):
        if self._h is None:
            raise Error(PETSC_ERR_ARG_WRONG, "Not for unassembled matrix")
        return self._h.info()

    def getSize(self):
        if self._h is None:
            return (self._size[1], self._size[3])
        i = self._info()
        return (i["M"], i["N"])

    def getLocalSize(self):
        i = self._info()
        return (i["m"], i["n"])

    def getSizes(self):
        i = self._info()
        return ((i["m"], i["M"]), (i["n"], i["N"]))

    def getOwnershipRange(self):
        i = self._info()
        return (i["rstart"], i["rstart"] + i["m"])

    def getOwnershipRangeColumn(self):
        i = self._info()
        return (i["cstart"], i["cstart"] + i["n"])

    def getType(self):
        return "mpiaij" if self._comm.size > 1 else "seqaij"

    def getComm(self):
        return self._comm

    size = property(getSize)
    local_size = property(getLocalSize)
    owner_range = property(getOwnershipRange)

    def getInfo(self, info=None):
        i = self._info()
        return {"nz_used": float(i["nnz_d"] + i["nnz_o"]), "nz_allocated": float(i["nnz_d"] + i["nnz_o"])}

    def getValuesCSR(self):
        """Local rows with GLOBAL sorted column ids (MatGetRow_MPIAIJ merge)."""
        ip, cj, vv = _guard(self._h.csr)
        return ip.astype(np.int32), cj.astype(np.int32), vv

    def getSplit(self):
        """The MPIAIJ split (A_d, A_o, garray) as stored on the device."""
        return _guard(self._h.split)

    def getVecs(self):
        """(right, left) vectors: x with the column layout, b with the row layout (test.py:29)."""
        return self.createVecRight(), self.createVecLeft()

    createVecs = getVecs

    def createVecRight(self):
        i = self._info()
        v = Vec()._setup(_mpi(self._comm), i["n"], i["N"])
        return v

    def createVecLeft(self):
        i = self._info()
        return Vec()._setup(_mpi(self._comm), i["m"], i["M"])

    getVecRight = createVecRight
    getVecLeft = createVecLeft

    def mult(self, x: Vec, y: Vec):
        self._dc.activate()
        _guard(self._h.mult, x._t, y._t)

    def multAdd(self, x: Vec, v2: Vec, v3: Vec):
        tmp = v3.duplicate()
        self.mult(x, tmp)
        if v3 is not v2:
            v2.copy(v3)
        v3.axpy(1.0, tmp)

    def getDiagonal(self, result: Vec = None):
        if result is None:
            result = self.createVecLeft()
        self._dc.activate()
        _guard(self._h.diagonal, result._t)
        return result

    def load(self, viewer):
        """MatLoad: the next AIJ matrix of a binary viewer, rows split by
        PetscSplitOwnership, assembled on the GPU."""
        from . import petsc_io
        M, N, ip, cj, vv = petsc_io.read_mat(viewer._fh)
        mc = _mpi(viewer._comm)
        r0, m = _split(M, mc.Get_size(), mc.Get_rank())
        lip = ip[r0:r0 + m + 1] - ip[r0]
        return self.createAIJ(size=(M, N), csr=(lip, cj[ip[r0]:ip[r0 + m]], vv[ip[r0]:ip[r0 + m]]), comm=mc)

    def view(self, viewer=None):
        if isinstance(viewer, Viewer):
            from . import petsc_io
            mc = _mpi(self._comm)
            part = self.getValuesCSR()
            parts = mc.allgather(part) if mc.Get_size() > 1 else [part]
            if mc.Get_rank() == 0:
                M, N = self.getSize()
                lens = np.concatenate([np.diff(p[0]) for p in parts])
                ip = np.concatenate([[0], np.cumsum(lens)])
                petsc_io.write_mat(viewer._fh, M, N, ip, np.concatenate([p[1] for p in parts]),
                                   np.concatenate([p[2] for p in parts]))
                viewer._fh.flush()
            return
        # PETSC_VIEWER_STDOUT_WORLD, default ASCII format (MatView_MPIAIJ gathers
        # the rows on rank 0, MatView_SeqAIJ_ASCII prints "row i: (j, v) ...")
        mc = _mpi(self._comm)
        part = self.getValuesCSR()
        parts = mc.allgather(part) if mc.Get_size() > 1 else [part]
        if mc.Get_rank() == 0:
            P = mc.Get_size()
            lines = [f"Mat Object: {P} MPI process{'es' if P > 1 else ''}", f"  type: {self.getType()}"]
            r = 0
            for ip, cj, vv in parts:
                for k in range(len(ip) - 1):
                    ents = "".join(f" ({int(cj[e])}, {_petsc_g(vv[e])}) " for e in range(ip[k], ip[k + 1]))
                    lines.append(f"row {r}:{ents}")
                    r += 1
            print("\n".join(lines), flush=True)

    def destroy(self):
        if self._h is not None:
            self._h.destroy()
            self._h = None
        return self

    def getDeviceHandle(self):
        return self._h


# ------------------------------------------------------------------ PC / KSP
class PC:
    class Type:
        NONE, JACOBI, LU, ILU, BJACOBI, SOR = "none", "jacobi", "lu", "ilu", "bjacobi", "sor"

    class Side:
        LEFT, RIGHT, SYMMETRIC = 0, 1, 2

    def __init__(self):
        self._type = None
        self._solver = None
        self._prefix = ""
        self._comm = None

    def create(self, comm=None):
        self._comm = Comm(_mpi(comm))
        return self

    def setType(self, t):
        self._type = str(t).lower()

    def getType(self):
        return self._type

    def setFactorSolverType(self, solver):
        self._solver = str(solver).lower()

    def getFactorSolverType(self):
        return self._solver

    def setFromOptions(self):
        o = Options(self._prefix)
        t = o.getString("pc_type")
        if t:
            self._type = t.lower()
        s = o.getString("pc_factor_mat_solver_type")
        if s:
            self._solver = s.lower()

    def setOptionsPrefix(self, p):
        self._prefix = p or ""

    def setUp(self):
        return self

    def destroy(self):
        return self


_REASON_NAMES = {2: "CONVERGED_RTOL", 3: "CONVERGED_ATOL", 4: "CONVERGED_ITS", 1: "CONVERGED_RTOL_NORMAL",
                 9: "CONVERGED_ATOL_NORMAL", 7: "CONVERGED_HAPPY_BREAKDOWN", -2: "DIVERGED_NULL",
                 -3: "DIVERGED_ITS", -4: "DIVERGED_DTOL", -5: "DIVERGED_BREAKDOWN",
                 -8: "DIVERGED_INDEFINITE_PC", -9: "DIVERGED_NANORINF", -10: "DIVERGED_INDEFINITE_MAT",
                 0: "CONVERGED_ITERATING"}


class KSP:
    class Type:
        CG, GMRES, PREONLY, RICHARDSON, BCGS, FGMRES = "cg", "gmres", "preonly", "richardson", "bcgs", "fgmres"

    class NormType:
        NONE, PRECONDITIONED, UNPRECONDITIONED, NATURAL, DEFAULT = 0, 1, 2, 3, -1
        NORM_NONE, NORM_PRECONDITIONED, NORM_UNPRECONDITIONED, NORM_NATURAL, NORM_DEFAULT = 0, 1, 2, 3, -1

    class ConvergedReason:
        CONVERGED_ITERATING = ITERATING = 0
        CONVERGED_RTOL_NORMAL = 1
        CONVERGED_RTOL = 2
        CONVERGED_ATOL = 3
        CONVERGED_ITS = 4
        CONVERGED_HAPPY_BREAKDOWN = 7
        DIVERGED_NULL = -2
        DIVERGED_ITS = -3
        DIVERGED_DTOL = -4
        DIVERGED_BREAKDOWN = -5
        DIVERGED_INDEFINITE_PC = -8
        DIVERGED_NANORINF = -9
        DIVERGED_INDEFINITE_MAT = -10
        DIVERGED_PC_FAILED = -11

    def __init__(self):
        self._type = None
        self._pc = PC()
        self._A = None
        self._comm = None
        self._rtol, self._atol, self._dtol, self._max_it = 1e-5, 1e-50, 1e5, 10000
        self._restart = 30
        self._norm = -1
        self._guess_nonzero = False
        self._its, self._reason, self._rnorm = 0, 0, 0.0
        self._history = None
        self._want_history = False
        self._prefix = ""
        self._flags = {}
        self._timing = {}

    def create(self, comm=None):
        self._comm = Comm(_mpi(comm))
        self._pc.create(comm)
        return self

    def setType(self, t):
        self._type = str(t).lower()

    def getType(self):
        return self._type or "gmres"

    def getPC(self):
        return self._pc

    def setPC(self, pc):
        self._pc = pc

    def setOperators(self, A, P=None):
        if A is not self._A:
            self._release_operator()
            if A is not None:
                # the solver state lives on the operator (mx_ksp.hip): count the
                # KSPs sharing it so one's reset leaves the others' state alone
                A._ksp_users = getattr(A, "_ksp_users", 0) + 1
        self._A = A

    def _release_operator(self):
        """This KSP stops using its operator; the last user releases the
        operator's solver state (KSPReset / KSPDestroy leave the Mat itself)."""
        A, self._A = self._A, None
        if A is None:
            return
        A._ksp_users = max(getattr(A, "_ksp_users", 1) - 1, 0)
        h = A.getDeviceHandle()
        if A._ksp_users == 0 and h is not None and h.h:
            _guard(h.ksp_reset)

    def getOperators(self):
        return self._A, self._A

    def setTolerances(self, rtol=None, atol=None, divtol=None, max_it=None):
        if rtol is not None and rtol != DEFAULT:
            self._rtol = float(rtol)
        if atol is not None and atol != DEFAULT:
            self._atol = float(atol)
        if divtol is not None and divtol != DEFAULT:
            self._dtol = float(divtol)
        if max_it is not None and max_it != DEFAULT:
            self._max_it = int(max_it)

    def getTolerances(self):
        return (self._rtol, self._atol, self._dtol, self._max_it)

    rtol = property(lambda s: s._rtol)
    atol = property(lambda s: s._atol)
    max_it = property(lambda s: s._max_it)

    def setGMRESRestart(self, restart):
        self._restart = int(restart)

    def setNormType(self, nt):
        self._norm = int(nt)

    def getNormType(self):
        return self._norm

    def setInitialGuessNonzero(self, flag):
        self._guess_nonzero = bool(flag)

    def getInitialGuessNonzero(self):
        return self._guess_nonzero

    def setConvergenceHistory(self, length=None, reset=False):
        self._want_history = True

    def getConvergenceHistory(self):
        return np.array([] if self._history is None else self._history)

    def setOptionsPrefix(self, prefix):
        self._prefix = prefix or ""
        self._pc.setOptionsPrefix(prefix)

    def getOptionsPrefix(self):
        return self._prefix

    def setFromOptions(self):
        """Options override explicit setters (test.py:46): -ksp_type, -pc_type,
        -ksp_rtol/atol/divtol/max_it, -ksp_gmres_restart, -ksp_norm_type,
        -ksp_initial_guess_nonzero, -ksp_monitor, -ksp_converged_reason, -ksp_view,
        -log_view, -ksp_error_if_not_converged."""
        o = Options(self._prefix)
        t = o.getString("ksp_type")
        if t:
            self._type = t.lower()
        self.setTolerances(o.getReal("ksp_rtol"), o.getReal("ksp_atol"), o.getReal("ksp_divtol"),
                           o.getInt("ksp_max_it"))
        r = o.getInt("ksp_gmres_restart")
        if r:
            self._restart = r
        nt = o.getString("ksp_norm_type")
        if nt:
            self._norm = {"none": 0, "preconditioned": 1, "unpreconditioned": 2, "natural": 3,
                          "default": -1}[nt.lower()]
        g = o.getBool("ksp_initial_guess_nonzero")
        if g is not None:
            self._guess_nonzero = g
        for f in ("ksp_monitor", "ksp_converged_reason", "ksp_view", "ksp_error_if_not_converged"):
            if o.hasName(f):
                self._flags[f] = o.getBool(f, True)
        self._flags["log_view"] = Options().hasName("log_view")
        self._pc.setFromOptions()

    def setUp(self):
        return self

    def _params(self):
        pct = (self._pc.getType() or ("jacobi" if self.getType() != "preonly" else "none"))
        return pct

    def solve(self, b: Vec, x: Vec):
        """KSPSolve (test.py:50) on the GPU."""
        if self._A is None:
            raise Error(PETSC_ERR_ARG_WRONG, "Must call KSPSetOperators() first")
        kt = self.getType()
        pct = self._params()
        if kt == "preonly" and pct == "lu":
            from . import direct
            t0 = time.perf_counter()
            _guard(direct.lu_solve, self._A, b, x)
            self._its, self._reason, self._rnorm = 1, 4, 0.0
            self._timing = {"KSPSolve": time.perf_counter() - t0}
            self._report()
            return
        if kt not in ("cg", "gmres", "preonly"):
            raise Error(PETSC_ERR_SUP, f"KSP type {kt} is not on the GPU path (cg, gmres, preonly)")
        if pct not in ("jacobi", "none"):
            raise Error(PETSC_ERR_SUP, f"PC type {pct} is not on the GPU path (jacobi, none; lu with preonly)")
        h = self._A.getDeviceHandle()
        self._A._dc.activate()
        t0 = time.perf_counter()
        r = _guard(h.solve, b._t, x._t, ksp=kt, pc=pct, rtol=self._rtol, atol=self._atol, dtol=self._dtol,
                   max_it=self._max_it, restart=self._restart,
                   norm={-1: "default", 0: "none", 1: "preconditioned", 2: "unpreconditioned", 3: "natural"}[self._norm],
                   guess_nonzero=self._guess_nonzero,
                   history=self._want_history or bool(self._flags.get("ksp_monitor")))
        self._timing = {"KSPSolve": time.perf_counter() - t0, "device_ms": r["solve_ms"]}
        self._its, self._reason, self._rnorm = r["its"], r["reason"], r["rnorm"]
        self._history = r.get("history")
        self._report()
        if self._reason < 0 and self._flags.get("ksp_error_if_not_converged"):
            raise Error(91, f"KSPSolve has not converged, reason {_REASON_NAMES.get(self._reason)}")

    def _report(self):
        rank0 = self._comm is None or self._comm.rank == 0
        if not rank0:
            return
        if self._flags.get("ksp_monitor") and self._history is not None:
            for i, v in enumerate(self._history):
                print(f"{i:3d} KSP Residual norm {v:14.12e}")
        if self._flags.get("ksp_converged_reason"):
            word = "converged" if self._reason > 0 else "did not converge"
            print(f"Linear solve {word} due to {_REASON_NAMES.get(self._reason, self._reason)} iterations {self._its}")
        if self._flags.get("ksp_view"):
            self.view()
        if self._flags.get("log_view"):
            print(f"KSPSolve: {self._timing.get('KSPSolve', 0.0):.6e} s wall, {self._its} its")

    def getIterationNumber(self):
        return self._its

    def getConvergedReason(self):
        return self._reason

    def getResidualNorm(self):
        return self._rnorm

    its = property(getIterationNumber)
    reason = property(getConvergedReason)
    norm = property(getResidualNorm)

    def view(self, viewer=None):
        print(f"KSP Object: {self._comm.size if self._comm else 1} MPI process(es)\n  type: {self.getType()}\n"
              f"  maximum iterations={self._max_it}, initial guess is {'nonzero' if self._guess_nonzero else 'zero'}\n"
              f"  tolerances: relative={self._rtol:g}, absolute={self._atol:g}, divergence={self._dtol:g}\n"
              f"PC Object:\n  type: {self._params()}")

    def reset(self):
        """KSPReset: the KSP drops its operator; the solver state kept on the
        operator (work space, device convergence state, captured CG graph,
        PCSetUp_Jacobi) is released when no other KSP uses it."""
        self._release_operator()
        return self

    def destroy(self):
        self.reset()
        return self


def init(args=None, comm=None):
    _init_options(args)


class Sys:
    @staticmethod
    def Print(*args, comm=None, **kw):
        if _MPI.COMM_WORLD.Get_rank() == 0:
            print(*args, **kw)

    @staticmethod
    def getVersion():
        return (3, 22, 0)


class Log:
    @staticmethod
    def begin():
        pass
