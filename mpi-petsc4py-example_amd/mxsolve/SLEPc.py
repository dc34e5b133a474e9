"""slepc4py-compatible EPS (petsc_funcs.py:13-20, test2.py:87-97).

Out of the hot-path scope but needed so that
`import petsc_funcs` works (petsc_funcs.py:2 imports SLEPc at module top) and
test2.py's call sequence returns eigenvalues.  Hermitian problems only
(EPS.ProblemType.HEP, which test2.py requests): a thick-restart Lanczos method
(the symmetric form of SLEPc's default Krylov-Schur) whose operator
applications, inner products and updates are libmxsolve.so calls on device
vectors; only the small projected eigenproblem (ncv x ncv) is solved on the
host, as SLEPc's DS object does.  Defaults follow SLEPc: nev = 1,
ncv = max(2 nev, nev + 15), tol = 1e-8, which = LARGEST_MAGNITUDE,
relative convergence test |r| / |theta| <= tol.
"""
from __future__ import annotations

import numpy as np

from . import PETSc as _P
from . import core


class EPS:
    class ProblemType:
        HEP, NHEP, GHEP, GNHEP, PGNHEP, GHIEP = 1, 2, 3, 4, 5, 6

    class Which:
        LARGEST_MAGNITUDE, SMALLEST_MAGNITUDE, LARGEST_REAL, SMALLEST_REAL = 1, 2, 3, 4

    class Type:
        KRYLOVSCHUR, LANCZOS, POWER = "krylovschur", "lanczos", "power"

    class ConvergedReason:
        CONVERGED_TOL, DIVERGED_ITS, CONVERGED_ITERATING = 1, -1, 0

    def __init__(self):
        self._A = None
        self._comm = None
        self._ptype = None
        self._nev, self._ncv, self._tol, self._max_it = 1, None, 1e-8, None
        self._which = EPS.Which.LARGEST_MAGNITUDE
        self._vals, self._vecs, self._its, self._reason = [], [], 0, 0
        self._prefix = ""

    def create(self, comm=None):
        self._comm = comm
        return self

    def setOperators(self, A, B=None):
        if B is not None:
            raise _P.Error(_P.PETSC_ERR_SUP, "generalized problems are not implemented")
        self._A = A

    def setProblemType(self, t):
        self._ptype = t

    def getProblemType(self):
        return self._ptype

    def setDimensions(self, nev=None, ncv=None, mpd=None):
        if nev is not None:
            self._nev = int(nev)
        if ncv is not None and ncv > 0:
            self._ncv = int(ncv)

    def getDimensions(self):
        return self._nev, self._ncv_eff(), self._ncv_eff()

    def setTolerances(self, tol=None, max_it=None):
        if tol is not None:
            self._tol = float(tol)
        if max_it is not None:
            self._max_it = int(max_it)

    def setWhichEigenpairs(self, w):
        self._which = w

    def setType(self, t):
        pass

    def setOptionsPrefix(self, p):
        self._prefix = p or ""

    def setFromOptions(self):
        o = _P.Options(self._prefix)
        nev = o.getInt("eps_nev")
        if nev:
            self._nev = nev
        ncv = o.getInt("eps_ncv")
        if ncv:
            self._ncv = ncv
        tol = o.getReal("eps_tol")
        if tol:
            self._tol = tol
        mi = o.getInt("eps_max_it")
        if mi:
            self._max_it = mi
        if o.hasName("eps_smallest_magnitude"):
            self._which = EPS.Which.SMALLEST_MAGNITUDE
        if o.hasName("eps_largest_real"):
            self._which = EPS.Which.LARGEST_REAL
        if o.hasName("eps_smallest_real"):
            self._which = EPS.Which.SMALLEST_REAL

    def _ncv_eff(self):
        N = self._A.getSize()[0]
        ncv = self._ncv or max(2 * self._nev, self._nev + 15)
        return min(ncv, N)

    def _order(self, theta):
        w = self._which
        if w == EPS.Which.LARGEST_MAGNITUDE:
            return np.argsort(-np.abs(theta), kind="stable")
        if w == EPS.Which.SMALLEST_MAGNITUDE:
            return np.argsort(np.abs(theta), kind="stable")
        if w == EPS.Which.LARGEST_REAL:
            return np.argsort(-theta, kind="stable")
        return np.argsort(theta, kind="stable")

    def solve(self):
        if self._ptype not in (None, EPS.ProblemType.HEP):
            raise _P.Error(_P.PETSC_ERR_SUP, "only Hermitian (HEP) problems are implemented")
        A = self._A
        dc = A._dc
        dc.activate()
        h = A.getDeviceHandle()
        N = A.getSize()[0]
        m = A.getLocalSize()[0]
        ncv = self._ncv_eff()
        nev = min(self._nev, ncv)
        max_it = self._max_it or max(100, 2 * N // max(ncv, 1))
        V = [dc.zeros(m) for _ in range(ncv + 1)]
        # deterministic start vector (SLEPc uses a random one)
        r0, _ = A.getOwnershipRange()
        core.rhs_hash(dc, r0, V[0])
        nrm = core.vnorm(dc, V[0])
        core.vscale(dc, 1.0 / nrm, V[0])
        T = np.zeros((ncv, ncv))
        k = 0                       # locked Ritz vectors carried over a restart
        beta_tail = None            # coupling row of the arrowhead after a restart
        w = dc.zeros(m)
        its = 0
        conv_vals, conv_vecs = [], []
        while its < max_it:
            its += 1
            for j in range(k, ncv):
                h.mult(V[j], w)
                # classical Gram-Schmidt against V[0..j], applied twice
                # (refinement; SLEPc's default BV orthogonalisation is CGS with
                # refinement): all j + 1 dots in one VecMDot pass over w, then
                # one VecMAXPY -- two host round trips per pass instead of two
                # per basis vector
                hcol = np.zeros(j + 1)
                for _ in range(2):
                    c = core.vmdot(dc, w, V[: j + 1])
                    hcol += c
                    core.vmaxpy(dc, w, -c, V[: j + 1])
                T[: j + 1, j] = hcol
                T[j, : j + 1] = hcol
                beta = core.vnorm(dc, w)
                if beta > 0:
                    V[j + 1].copy_(w)
                    core.vscale(dc, 1.0 / beta, V[j + 1])
                if j + 1 < ncv:
                    T[j + 1, j] = T[j, j + 1] = beta
                last_beta = beta
            Ts = 0.5 * (T + T.T)
            theta, S = np.linalg.eigh(Ts)
            order = self._order(theta)
            theta, S = theta[order], S[:, order]
            res = np.abs(last_beta * S[-1, :])
            ok = res <= self._tol * np.maximum(np.abs(theta), 1e-300)
            nconv = 0
            while nconv < ncv and ok[nconv]:
                nconv += 1
            if nconv >= nev or its >= max_it:
                conv_vals = list(theta[:max(nconv, 0)])
                conv_vecs = S[:, :nconv]
                break
            # thick restart: keep the leading half of the Ritz vectors
            k = max(nev, ncv // 2)
            Y = [dc.zeros(m) for _ in range(k)]
            for q in range(k):
                core.vmaxpy(dc, Y[q], S[:ncv, q], V[:ncv])
            for q in range(k):
                V[q].copy_(Y[q])
            V[k].copy_(V[ncv])
            T = np.zeros((ncv, ncv))
            for q in range(k):
                T[q, q] = theta[q]
                T[q, k] = T[k, q] = last_beta * S[-1, q]
        self._its = its
        self._reason = EPS.ConvergedReason.CONVERGED_TOL if len(conv_vals) >= nev else EPS.ConvergedReason.DIVERGED_ITS
        self._vals = conv_vals
        self._basis = V[:ncv]
        self._S = conv_vecs

    def getConverged(self):
        return len(self._vals)

    def getIterationNumber(self):
        return self._its

    def getConvergedReason(self):
        return self._reason

    def getEigenvalue(self, i):
        return float(self._vals[i])

    def getEigenpair(self, i, Vr=None, Vi=None):
        if Vr is not None:
            dc = self._A._dc
            dc.activate()
            Vr._t.zero_()
            for j, v in enumerate(self._basis):
                core.vaxpy(dc, self._S[j, i], v, Vr._t)
        if Vi is not None:
            Vi.set(0.0)
        return float(self._vals[i])

    def destroy(self):
        return self
