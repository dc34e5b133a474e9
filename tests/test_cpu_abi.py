"""The C-ABI library loads here (no GPU) and exports every symbol include/mxsolve.h declares."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mxsolve.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mx_[a-z0-9_]+)\s*\(", src)))


def test_header_lists_the_abi():
    syms = header_symbols()
    for s in ("mx_mat_create_csr", "mx_mat_mult", "mx_ksp_solve", "mx_comm_create_rccl", "mx_vec_dot"):
        assert s in syms


def test_library_exports_every_symbol():
    from mxsolve import _lib
    L = _lib.load()
    for s in header_symbols():
        assert hasattr(L, s), s
    assert set(header_symbols()) == set(_lib.SIGNATURES), "ctypes signature table out of sync with the header"


def test_cpu_only_calls():
    import ctypes as C
    from mxsolve import _lib
    L = _lib.load()
    assert L.mx_version() == 3
    r = (C.c_int64 * 5)()
    assert L.mx_layout_split(10, 4, r) == 0 and list(r) == [0, 3, 6, 8, 10]
    p = _lib.KSPParams()
    L.mx_ksp_default_params(C.byref(p))
    assert (p.max_it, p.restart, p.rtol, p.atol, p.dtol) == (10000, 30, 1e-5, 1e-50, 1e5)


def test_no_gpu_fails_loudly():
    """Without a GPU the product path raises (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mxsolve import _lib
    from mxsolve.core import DeviceComm
    with pytest.raises((_lib.MxError, RuntimeError)):
        DeviceComm.self_comm(0)


def test_built_for_gfx950():
    """The fat binary embeds a gfx950 code object (and no other GPU target)."""
    so = os.path.join(ROOT, "mpi-petsc4py-example_amd", "lib", "libmxsolve.so")
    data = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_every_debug_key_documented():
    """Every measurement knob mx_debug_set accepts (csrc/mx_abi.hip) has its
    "key N:" entry in include/mxsolve.h, so an A/B setting named in DESIGN.md
    or a profile can be looked up."""
    import re
    abi = open(os.path.join(ROOT, "mpi-petsc4py-example_amd", "csrc", "mx_abi.hip")).read()
    keys = sorted({int(k) for k in re.findall(r"case (\d+): old = g_knobs", abi)})
    hdr = open(os.path.join(ROOT, "include", "mxsolve.h")).read()
    doc = {int(k) for k in re.findall(r"key (\d+):", hdr)}
    assert keys and not [k for k in keys if k not in doc]
