"""Value codes: a diagonal block with at most 256 distinct values streams one
byte per slot into an LDS value table (mx_assembly.hip build_value_codes).
The product must stay bit-identical to the oracle, with codes, without them
(more distinct values, or knob 23 = 0), on aligned-offset slices of every
width class (fixed 5/7/27, runtime k, k > 8 = several code batches, odd k)
and on general SELL slices (column ids + codes, odd widths)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def lib():
    from mxsolve import _lib
    return _lib.load()


def mult_bits(comm, oracle_mod, M, ip, c, v, seed=3):
    from mxsolve.core import DMat
    A = DMat.from_csr(comm, M, M, ip, c, v)
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    x = np.random.default_rng(seed).standard_normal(M)
    y = torch.zeros(M, dtype=torch.float64, device="cuda")
    A.mult(torch.from_numpy(x).cuda(), y)
    got = y.cpu().numpy().view(np.uint64)
    return A.info(), got, O.mult(x).view(np.uint64)


def banded(M, offsets, values, rng, drop=0.0):
    """Rows with the given column offsets (clipped at the edges, some dropped)."""
    ip, cols, vals = [0], [], []
    for i in range(M):
        for o in offsets:
            j = i + o
            if 0 <= j < M and (o == 0 or rng.random() >= drop):
                cols.append(j)
                vals.append(values[rng.integers(0, len(values))])
        ip.append(len(cols))
    return np.array(ip, np.int64), np.array(cols, np.int64), np.array(vals)


@pytest.mark.parametrize("kind,n", [("poisson2d", 37), ("poisson3d", 19), ("poisson3d27", 9), ("convdiff3d", 13)])
def test_stencils_use_codes(selfcomm, oracle_mod, kind, n):
    ip, c, v = oracle_mod.stencil(kind, n)
    info, got, exp = mult_bits(selfcomm, oracle_mod, ip.size - 1, ip, c, v)
    assert 0 < info["value_codes"] <= 256
    assert info["code_bytes"] > 0
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("offsets", [
    (-3, -1, 0, 1, 3),                              # k = 5 (fixed body)
    (-40, -7, -1, 0, 1, 7, 40),                     # k = 7
    (-2, -1, 0, 1, 2, 5),                           # k = 6 (runtime body, one batch)
    tuple(range(-6, 7)),                            # k = 13: two batches, odd
    tuple(range(-8, 9)),                            # k = 17: three batches
    tuple(range(-16, 16)),                          # k = 32 = DIA_MAX: every mask bit, a full LDS image
    tuple(range(-16, 17)),                          # k = 33: past DIA_MAX, general slices
])
@pytest.mark.parametrize("nvals", [1, 3, 255])
def test_aligned_offset_slices(selfcomm, oracle_mod, offsets, nvals):
    rng = np.random.default_rng(len(offsets) * 1000 + nvals)
    values = np.unique(rng.standard_normal(nvals)) if nvals > 1 else np.array([-1.0])
    assert values.size == nvals
    ip, c, v = banded(1000, offsets, values, rng, drop=0.1)
    info, got, exp = mult_bits(selfcomm, oracle_mod, 1000, ip, c, v)
    assert info["value_codes"] == np.unique(v.view(np.uint64)).size   # stored values only
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("maxlen", [3, 9, 40])
def test_general_slices(selfcomm, oracle_mod, maxlen):
    """Irregular rows (general SELL, column ids) with few distinct values,
    signed zeros among them."""
    rng = np.random.default_rng(maxlen)
    M = 777
    lens = rng.integers(0, maxlen + 1, M)
    ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    cols = np.concatenate([np.sort(rng.choice(M, size=k, replace=False)) for k in lens]).astype(np.int64)
    vals = np.array([0.5, -2.0, 0.0, -0.0, 3.25, 1e300])[rng.integers(0, 6, cols.size)]
    info, got, exp = mult_bits(selfcomm, oracle_mod, M, ip, cols, vals)
    assert info["value_codes"] > 0
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("nvals,coded", [(255, True), (256, False)])
def test_table_limit(selfcomm, oracle_mod, nvals, coded):
    """255 distinct values fit (code 255 marks absent slots), 256 do not."""
    rng = np.random.default_rng(nvals)
    values = np.unique(rng.standard_normal(nvals))
    ip, c, v = banded(3000, (-2, -1, 0, 1, 2), values, rng, drop=0.05)
    v[: values.size] = values                     # every value stored at least once
    info, got, exp = mult_bits(selfcomm, oracle_mod, 3000, ip, c, v)
    assert (info["value_codes"] == nvals) if coded else (info["value_codes"] == 0)
    assert np.array_equal(got, exp)


def test_too_many_values_falls_back(selfcomm, oracle_mod):
    rng = np.random.default_rng(5)
    values = np.unique(rng.standard_normal(400))
    ip, c, v = banded(2000, (-1, 0, 1), values, rng)
    assert np.unique(v).size > 256
    info, got, exp = mult_bits(selfcomm, oracle_mod, 2000, ip, c, v)
    assert info["value_codes"] == 0
    assert np.array_equal(got, exp)


def test_knob_off_same_bits(selfcomm, oracle_mod):
    ip, c, v = oracle_mod.stencil("convdiff3d", 12)
    L = lib()
    old = L.mx_debug_set(23, 0)
    try:
        info0, got0, exp = mult_bits(selfcomm, oracle_mod, ip.size - 1, ip, c, v)
    finally:
        L.mx_debug_set(23, old)
    info1, got1, _ = mult_bits(selfcomm, oracle_mod, ip.size - 1, ip, c, v)
    assert info0["value_codes"] == 0 and info1["value_codes"] > 0
    assert np.array_equal(got0, exp) and np.array_equal(got1, exp)


def test_cg_with_and_without_codes(selfcomm):
    """The whole CG solve: same iteration count and the same solution bits."""
    from mxsolve.core import DMat, rhs_hash
    L = lib()
    res = []
    old27 = L.mx_debug_set(27, 0)          # single-row layout in both (same dot grouping)
    old43 = L.mx_debug_set(43, 0)          # and the same (resident) grid for the fp64 values
    for knob in (0, 1):
        old = L.mx_debug_set(23, knob)
        try:
            A = DMat.stencil(selfcomm, "poisson3d", 32)
            m = A.info()["m"]
            b = selfcomm.empty(m)
            rhs_hash(selfcomm, 0, b)
            x = selfcomm.zeros(m)
            r = A.solve(b, x, ksp="cg", rtol=1e-8)
            res.append((r["its"], r["reason"], x.cpu().numpy().copy(), A.info()["value_codes"]))
        finally:
            L.mx_debug_set(23, old)
    L.mx_debug_set(27, old27)
    L.mx_debug_set(43, old43)
    assert res[0][3] == 0 and res[1][3] > 0
    assert res[0][:2] == res[1][:2]
    assert np.array_equal(res[0][2].view(np.uint64), res[1][2].view(np.uint64))


@pytest.mark.parametrize("kind,n,shape", [("poisson2d", 38, 5), ("poisson3d", 24, 7), ("poisson3d27", 24, 27),
                                          ("convdiff3d", 12, 7), ("poisson3d", 19, 0)])
def test_row_pairs(selfcomm, oracle_mod, kind, n, shape):
    """Row-pair layout (even stencil offsets): MatMult bit-exact with pairs on
    and off; n = 19 (odd offsets) keeps the single-row layout."""
    ip, c, v = oracle_mod.stencil(kind, n)
    L = lib()
    old = L.mx_debug_set(27, 0)
    try:
        info0, got0, exp = mult_bits(selfcomm, oracle_mod, ip.size - 1, ip, c, v, seed=11)
    finally:
        L.mx_debug_set(27, old)
    info1, got1, _ = mult_bits(selfcomm, oracle_mod, ip.size - 1, ip, c, v, seed=11)
    assert info0["pair_shape"] == 0 and info1["pair_shape"] == shape
    assert np.array_equal(got0, exp) and np.array_equal(got1, exp)


@pytest.mark.parametrize("kind,n,ksp", [("poisson3d", 24, "cg"), ("poisson3d27", 24, "cg"),
                                        ("poisson2d", 38, "cg"), ("convdiff3d", 12, "gmres")])
def test_row_pairs_solve(selfcomm, oracle_mod, kind, n, ksp):
    """CG (MatMult + dot) and GMRES (Jacobi-scaled, lazily normalised operand)
    on the row-pair path against the oracle."""
    from mxsolve.core import DMat
    ip, c, v = oracle_mod.stencil(kind, n)
    M = ip.size - 1
    A = DMat.from_csr(selfcomm, M, M, ip, c, v)
    assert A.info()["pair_shape"] > 0
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    b = np.random.default_rng(5).random(M)
    bt = torch.from_numpy(b).cuda()
    x = torch.zeros(M, dtype=torch.float64, device="cuda")
    r = A.solve(bt, x, ksp=ksp, rtol=1e-8)
    o = O.solve(b, ksp=ksp, rtol=1e-8)
    assert r["reason"] == o["reason"] and abs(r["its"] - o["its"]) <= 1
    xs = x.cpu().numpy()
    assert np.linalg.norm(xs - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])


def _with_knob(L, key, value, fn):
    old = L.mx_debug_set(key, value)
    try:
        return fn()
    finally:
        L.mx_debug_set(key, old)


@pytest.mark.parametrize("kind,n,shape", [("poisson2d", 256, 5), ("poisson3d", 64, 7), ("poisson3d27", 48, 27),
                                          ("convdiff3d", 64, 7)])
def test_pair_code_dictionary(selfcomm, oracle_mod, kind, n, shape):
    """Row-pair code blocks deduplicated into a dictionary: a few distinct
    blocks, MatMult bit-exact against the oracle.  (The per-unit layout and
    the forced-collision check of rounds 3-5, knob 30, are retired.)"""
    ip, c, v = oracle_mod.stencil(kind, n)
    M = ip.size - 1
    info1, got1, exp = mult_bits(selfcomm, oracle_mod, M, ip, c, v, seed=13)
    assert info1["pair_shape"] == shape
    assert 0 < info1["pair_blocks"] <= info1["pair_units"] // 4
    assert np.array_equal(got1, exp)


@pytest.mark.parametrize("kind,n,shape,uni", [("poisson2d", 256, 5, 1), ("poisson3d", 64, 7, 1),
                                              ("poisson3d", 32, 7, 1), ("convdiff3d", 64, 7, 0)])
def test_pair_uniform_blocks(selfcomm, oracle_mod, kind, n, shape, uni):
    """Uniform-slot dictionary blocks (each block's slot values and lane masks
    read by scalar loads, no code bytes): MatMult bit-exact against the
    oracle.  The convection-diffusion operator's face coefficients vary along
    x, so its blocks are not uniform (the LDS-table path); nor is a dictionary
    whose slot-row holds two values."""
    ip, c, v = oracle_mod.stencil(kind, n)
    M = ip.size - 1
    info1, got1, exp = mult_bits(selfcomm, oracle_mod, M, ip, c, v, seed=17)
    assert info1["pair_shape"] == shape and info1["pair_blocks"] > 0 and info1["pair_uniform"] == uni
    assert np.array_equal(got1, exp)
    # two values in the diagonal slot-row of the interior units: not uniform
    v2 = v.copy()
    rows = np.repeat(np.arange(M), np.diff(ip))
    diag = (c == rows) & (rows % 3 == 0)
    v2[diag] *= 2.0
    info2, got2, exp2 = mult_bits(selfcomm, oracle_mod, M, ip, c, v2, seed=17)
    assert info2["pair_uniform"] == 0 and np.array_equal(got2, exp2)


@pytest.mark.parametrize("kind,n,ksp", [("convdiff3d", 24, "gmres"), ("poisson3d27", 16, "gmres")])
def test_pair_jacobi_by_code(selfcomm, oracle_mod, kind, n, ksp):
    """GMRES(30) + vector Jacobi on the row-pair path, dinv from the table
    indexed by the rows' diagonal code: iterations, reason and solution
    against the oracle."""
    from mxsolve.core import DMat
    ip, c, v = oracle_mod.stencil(kind, n)
    M = ip.size - 1
    L = lib()
    b = np.random.default_rng(9).random(M)

    def run():
        A = DMat.from_csr(selfcomm, M, M, ip, c, v)
        assert A.info()["pair_shape"] > 0
        bt = torch.from_numpy(b).cuda()
        x = torch.zeros(M, dtype=torch.float64, device="cuda")
        r = A.solve(bt, x, ksp=ksp, rtol=1e-8, history=True)
        A.destroy()
        return r["its"], r["reason"], r["history"].copy(), x.cpu().numpy().copy()

    on = run()
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    o = O.solve(b, ksp=ksp, rtol=1e-8)
    assert on[1] == o["reason"] and abs(on[0] - o["its"]) <= 1
    assert np.linalg.norm(on[3] - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])


def _with_knobs(L, kv, fn):
    """fn() under the knob settings kv ({key: value}), restored after."""
    old = {k: L.mx_debug_set(k, v) for k, v in kv.items()}
    try:
        return fn()
    finally:
        for k, v in old.items():
            L.mx_debug_set(k, v)


# lean-kernel forms: default (z-march, two planes per step, 4 workgroups per
# CU, segments of up to 32 planes), the sweep form (39 = 0), short / odd
# segments with tails (41), other grids (40) -- and for the 27-point z-march:
# its per-run-branch body instead of the column-zeroed one (48 = 0),
# multiply-and-add for the -1 slots instead of their exact-product fma (53 = 0),
# the carried-operand body instead of the plane-pipelined one (60 = 0).
# (The plane-step and 27-point grid variants, keys 42 / 49 / 45, are fixed
# since round 6.)
LEAN_FORMS = [{}, {39: 0}, {41: 3}, {41: 1, 40: 1}, {41: 5, 40: 3}, {40: 2},
              {48: 0}, {48: 0, 41: 5}, {53: 0}, {60: 0}, {60: 0, 53: 0}]


@pytest.mark.parametrize("form", range(len(LEAN_FORMS)))
@pytest.mark.parametrize("kind,n,lean", [("poisson3d", 128, 2), ("poisson2d", 256, 2), ("poisson2d", 384, 2),
                                         ("poisson3d", 64, 1), ("poisson2d", 96, 1), ("poisson3d", 48, 1),
                                         ("poisson3d27", 128, 2), ("poisson3d27", 64, 1)])
def test_pair_lean_kernel(selfcomm, oracle_mod, kind, n, lean, form):
    """Lean row-pair MatMult (mx_spmv_pair.hip, knob 38 = 1, the default) for
    uniform-slot layouts: bit-exact against the oracle and against the general
    SELL kernel (knob 38 = 0).  lean = 2: every block select-free (absent
    operands read as 0.0 -- y/z-boundary runs and the x-line edges, x-lines a
    multiple of 128 rows); lean = 1: a block whose -1/+1 slot-row misses a lane
    other than the unit's edge lane (x-lines of 64 / 96 / 48 rows inside a
    128-row unit) keeps the presence selects.
    The 27-point operator has the z-march form only (nine runs, six carried);
    its clean layout skips a unit's empty runs by a wave-uniform branch, the
    other layout selects by the lane's transposed mask bits.
    Operand values include infinities and NaN: an absent slot must not let them
    into a row that PETSc's product keeps finite."""
    ip, c, v = oracle_mod.stencil(kind, n)
    M = ip.size - 1
    L = lib()
    from mxsolve.core import DMat
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    rng = np.random.default_rng(23)
    for special in (False, True):
        x = rng.standard_normal(M)
        if special:
            x[rng.integers(0, M, 40)] = np.inf
            x[rng.integers(0, M, 40)] = -np.inf
            x[rng.integers(0, M, 40)] = np.nan
        exp = O.mult(x).view(np.uint64)
        outs = []
        for knob in (1, 0):
            def run():
                A = DMat.from_csr(selfcomm, M, M, ip, c, v)
                y = torch.zeros(M, dtype=torch.float64, device="cuda")
                A.mult(torch.from_numpy(x).cuda(), y)
                info = A.info()
                A.destroy()
                return info, y.cpu().numpy().view(np.uint64)
            outs.append(_with_knobs(L, {38: knob, **LEAN_FORMS[form]}, run))
        (i1, g1), (i0, g0) = outs
        # the 27-point lean kernel exists as a z-march only (knob 39 = 0: the general kernel)
        exp_lean = 0 if kind == "poisson3d27" and LEAN_FORMS[form].get(39) == 0 else lean
        assert i1["pair_uniform"] == 1 and i1["pair_lean"] == exp_lean and i0["pair_lean"] == 0
        if kind == "poisson3d27" and exp_lean:
            # a clean layout gets the column words unless knob 48 = 0; the other keeps the selects
            assert i1["pair_form27"] == (0 if lean == 1 else 1 if LEAN_FORMS[form].get(48) == 0 else 2)
        assert np.array_equal(g1, exp) and np.array_equal(g0, exp)


@pytest.mark.parametrize("n", [128, 96])
def test_pair_lean_cg(selfcomm, oracle_mod, n):
    """CG with the lean MatMult (+ p.w partials) and with the general kernel.
    The sweep form (knob 39 = 0) walks the general kernel's grid and order:
    same iterations, history and solution bits.  The z-march form groups each
    lane's p.w terms by column, not by sweep step: same iterations and reason,
    iterates equal to rounding; both against the oracle."""
    from mxsolve.core import DMat, rhs_hash
    L = lib()

    def run():
        A = DMat.stencil(selfcomm, "poisson3d" if n == 128 else "poisson2d", n)
        m = A.info()["m"]
        b = selfcomm.empty(m)
        rhs_hash(selfcomm, 0, b)
        x = selfcomm.zeros(m)
        r = A.solve(b, x, ksp="cg", pc="jacobi", history=True)
        kind = A.info()["pair_lean"]
        A.destroy()
        return r["its"], r["reason"], r["history"].copy(), x.cpu().numpy().copy(), kind

    zm = run()
    sweep = _with_knob(L, 39, 0, run)
    off = _with_knob(L, 38, 0, run)
    assert zm[4] > 0 and sweep[4] > 0 and off[4] == 0
    assert sweep[:2] == off[:2]
    assert np.array_equal(sweep[2].view(np.uint64), off[2].view(np.uint64))
    assert np.array_equal(sweep[3].view(np.uint64), off[3].view(np.uint64))
    assert zm[:2] == off[:2]
    assert np.allclose(zm[2], off[2], rtol=1e-9, atol=0)
    assert np.linalg.norm(zm[3] - off[3]) <= 1e-10 * np.linalg.norm(off[3])


@pytest.mark.parametrize("kind,n,f64", [("poisson3d", 128, 7), ("poisson2d", 256, 5), ("poisson3d", 64, 0)])
def test_pair_f64_zmarch(selfcomm, oracle_mod, kind, n, f64):
    """fp64-valued (uncoded: every entry a different value) 5/7-point blocks
    get an fp64 row-pair layout and the z-march MatMult (knob 44 = 1, the
    default) when every unit is select-free (x-lines a multiple of 128 rows;
    64-row lines keep the aligned-offset SELL kernel): MatMult bit-exact
    against the oracle and against knob 44 = 0, operands with infinities and
    NaN included; CG on the symmetrically scaled operator D A D against the
    oracle."""
    from mxsolve.core import DMat
    ip, c, v = oracle_mod.stencil(kind, n)
    M = ip.size - 1
    rng = np.random.default_rng(29)
    f = 1.0 + 0.5 * rng.random(M)
    rows = np.repeat(np.arange(M), np.diff(ip))
    v = v * f[rows] * f[c]                         # D A D: SPD, ~all values distinct
    L = lib()
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    for special in (False, True):
        x = rng.standard_normal(M)
        if special:
            x[rng.integers(0, M, 40)] = np.inf
            x[rng.integers(0, M, 40)] = -np.inf
            x[rng.integers(0, M, 40)] = np.nan
        exp = O.mult(x).view(np.uint64)
        A = DMat.from_csr(selfcomm, M, M, ip, c, v)
        y = torch.zeros(M, dtype=torch.float64, device="cuda")
        A.mult(torch.from_numpy(x).cuda(), y)
        i1 = A.info()
        A.destroy()
        g1 = y.cpu().numpy().view(np.uint64)
        assert i1["value_codes"] == 0 and i1["pair_f64"] == f64
        assert np.array_equal(g1, exp)
    A = DMat.from_csr(selfcomm, M, M, ip, c, v)
    b = rng.random(M)
    xs = torch.zeros(M, dtype=torch.float64, device="cuda")
    r = A.solve(torch.from_numpy(b).cuda(), xs, ksp="cg", rtol=1e-8)
    A.destroy()
    o = O.solve(b, ksp="cg", rtol=1e-8)
    assert r["reason"] == o["reason"] and abs(r["its"] - o["its"]) <= 1
    assert np.linalg.norm(xs.cpu().numpy() - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])


def _periodic_2d(oracle_mod, n):
    """2D 5-point operator with row scales of period 4 in x (four distinct row
    factors): a code dictionary that is not uniform per slot-row (a slot's
    value differs between lanes), nonsymmetric."""
    ip, c, v = oracle_mod.stencil("poisson2d", n)
    M = ip.size - 1
    f = np.array([1.0, 1.25, 1.5, 2.0])[np.arange(M) % n % 4]
    rows = np.repeat(np.arange(M), np.diff(ip))
    return ip, c, v * f[rows]


ZMC_FORMS = [{}, {41: 3}, {41: 1, 40: 1}, {41: 5, 40: 3}]


@pytest.mark.parametrize("form", range(len(ZMC_FORMS)))
@pytest.mark.parametrize("kind,n,applies", [("convdiff3d", 128, 1), ("periodic2d", 256, 1), ("convdiff3d", 64, 0)])
def test_pair_code_zmarch(selfcomm, oracle_mod, kind, n, applies, form):
    """Coded z-march MatMult (spmv_pair_zmc_kernel, knob 52 = 1, the default)
    for 5/7-point code dictionaries that are not uniform per slot-row --
    BASELINE C4's convection-diffusion operator (kappa of period 4 in x) and a
    periodic-coefficient 2D operator: bit-exact against the oracle and against
    the general SELL kernel (knob 52 = 0), operands with infinities and NaN
    included, in every z-march form.  x-lines of 64 rows (not select-free)
    keep the general kernel (mx_mat_info.pair_code = 0)."""
    from mxsolve.core import DMat, dispatch_counts
    ip, c, v = _periodic_2d(oracle_mod, n) if kind == "periodic2d" else oracle_mod.stencil(kind, n)
    M = ip.size - 1
    L = lib()
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    rng = np.random.default_rng(37)
    for special in (False, True):
        x = rng.standard_normal(M)
        if special:
            x[rng.integers(0, M, 40)] = np.inf
            x[rng.integers(0, M, 40)] = -np.inf
            x[rng.integers(0, M, 40)] = np.nan
        exp = O.mult(x).view(np.uint64)
        outs = []
        for knob in (1, 0):
            def run():
                A = DMat.from_csr(selfcomm, M, M, ip, c, v)
                y = torch.zeros(M, dtype=torch.float64, device="cuda")
                dispatch_counts(reset=True)
                A.mult(torch.from_numpy(x).cuda(), y)
                dc = dispatch_counts(reset=True)
                info = A.info()
                A.destroy()
                return info, y.cpu().numpy().view(np.uint64), dc
            outs.append(_with_knobs(L, {52: knob, **ZMC_FORMS[form]}, run))
        (i1, g1, d1), (i0, g0, d0) = outs
        assert i1["pair_uniform"] == 0 and i1["pair_code"] == applies and i0["pair_code"] == 0
        assert d1["pair_zmc"] == applies and d0["pair_zmc"] == 0
        assert np.array_equal(g1, exp) and np.array_equal(g0, exp)


@pytest.mark.parametrize("kind,n,pc", [("convdiff3d", 128, "jacobi"), ("periodic2d", 256, "none"),
                                       ("periodic2d", 512, "jacobi")])
def test_pair_code_zmarch_gmres(selfcomm, oracle_mod, kind, n, pc):
    """GMRES(30) on the coded z-march: its MatMult forms the operand fl(s x)
    of the unnormalised basis vector and applies Jacobi by the diagonal code
    (JACOBI_S) or nothing (PLAIN_S).  The same per-row sums as the general
    kernel, so the whole solve -- iterations, history, solution -- is bitwise
    that of knob 52 = 0; both against the oracle."""
    from mxsolve.core import DMat, dispatch_counts
    ip, c, v = _periodic_2d(oracle_mod, n) if kind == "periodic2d" else oracle_mod.stencil(kind, n)
    M = ip.size - 1
    L = lib()
    b = np.random.default_rng(41).random(M)

    def run():
        A = DMat.from_csr(selfcomm, M, M, ip, c, v)
        bt = torch.from_numpy(b).cuda()
        x = torch.zeros(M, dtype=torch.float64, device="cuda")
        dispatch_counts(reset=True)
        r = A.solve(bt, x, ksp="gmres", pc=pc, rtol=1e-8, max_it=400, history=True)
        dc = dispatch_counts(reset=True)
        A.destroy()
        return r["its"], r["reason"], r["history"].copy(), x.cpu().numpy().copy(), dc

    on = run()
    off = _with_knob(L, 52, 0, run)
    assert on[4]["pair_zmc"] >= on[0] and off[4]["pair_zmc"] == 0
    assert on[:2] == off[:2]
    assert np.array_equal(on[2].view(np.uint64), off[2].view(np.uint64))
    assert np.array_equal(on[3].view(np.uint64), off[3].view(np.uint64))
    O = oracle_mod.OracleMat.from_csr(M, M, ip, c, v)
    from _hostinfo import host_threads
    o = O.solve(b, ksp="gmres", pc=pc, rtol=1e-8, max_it=400, nthreads=host_threads())
    assert on[1] == o["reason"] and abs(on[0] - o["its"]) <= 1
    assert np.linalg.norm(on[3] - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])
