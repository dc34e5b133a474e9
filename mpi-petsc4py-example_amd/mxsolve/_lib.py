"""ctypes binding of libmxsolve.so (include/mxsolve.h).

The library is the only compute path: if it is missing or fails to load, every
operation raises -- there is no CPU fallback.  torch is imported first so that
libmxsolve.so binds to the HIP runtime torch already loaded (both carry the
SONAME libamdhip64.so.7): device pointers from torch tensors and from the
library then belong to one runtime.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (loads the process's HIP runtime before libmxsolve)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MXSOLVE_LIB", os.path.join(PKG_ROOT, "lib", "libmxsolve.so"))

MX_OK, MX_ERR_ARG, MX_ERR_OUTOFRANGE, MX_ERR_HIP, MX_ERR_COMM, MX_ERR_MEM, MX_ERR_UNSUPPORTED, MX_ERR_INTERNAL = range(8)
ERR_NAMES = {1: "ARG", 2: "OUTOFRANGE", 3: "HIP", 4: "COMM", 5: "MEM", 6: "UNSUPPORTED", 7: "INTERNAL"}


class MxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[mxsolve {ERR_NAMES.get(code, code)}] {msg}")
        self.code = code
        self.msg = msg


class KSPParams(C.Structure):
    _fields_ = [("ksp_type", C.c_int), ("pc_type", C.c_int), ("norm_type", C.c_int),
                ("max_it", C.c_int), ("restart", C.c_int), ("guess_nonzero", C.c_int),
                ("rtol", C.c_double), ("atol", C.c_double), ("dtol", C.c_double),
                ("haptol", C.c_double), ("breakdowntol", C.c_double),
                ("poll_every", C.c_int), ("profile", C.c_int)]


class KSPResult(C.Structure):
    _fields_ = [("its", C.c_int), ("reason", C.c_int), ("rnorm", C.c_double),
                ("solve_ms", C.c_double), ("spmv_ms", C.c_double), ("spmv_count", C.c_int),
                ("launched_its", C.c_int), ("cg_mode", C.c_int), ("upd_ms", C.c_double), ("upd_count", C.c_int),
                ("cg_xbatch", C.c_int), ("pb_ms", C.c_double), ("pb_count", C.c_int),
                ("pbw_ms", C.c_double), ("pbw_count", C.c_int), ("mdot_ms", C.c_double), ("mdot_count", C.c_int),
                ("maxpy_ms", C.c_double), ("maxpy_count", C.c_int)]


class MatInfo(C.Structure):
    _fields_ = [("M", C.c_int64), ("N", C.c_int64), ("m", C.c_int64), ("n", C.c_int64),
                ("rstart", C.c_int64), ("cstart", C.c_int64), ("nnz_d", C.c_int64),
                ("nnz_o", C.c_int64), ("nghost", C.c_int64), ("sell_slots_d", C.c_int64),
                ("sell_slots_o", C.c_int64), ("nsend_peers", C.c_int), ("nrecv_peers", C.c_int),
                ("nsend", C.c_int64), ("nrecv", C.c_int64), ("dia_slices", C.c_int64),
                ("value_codes", C.c_int64), ("code_bytes", C.c_int64), ("pair_shape", C.c_int64),
                ("pair_units", C.c_int64), ("pair_blocks", C.c_int64), ("pair_block_bytes", C.c_int64),
                ("pair_uniform", C.c_int64), ("pair_lean", C.c_int64),
                ("pair_zmarch", C.c_int64), ("pair_f64", C.c_int64), ("pair_form27", C.c_int64),
                ("pair_code", C.c_int64), ("cb_blocks", C.c_int64)]


P = C.c_void_p
I64 = C.c_int64
I64P = C.POINTER(C.c_int64)
DP = C.POINTER(C.c_double)

# name -> (restype, argtypes); every function in include/mxsolve.h
SIGNATURES = {
    "mx_version": (C.c_int, []),
    "mx_last_error": (C.c_int, [C.c_char_p, C.c_size_t]),
    "mx_get_unique_id": (C.c_int, [P, C.c_size_t]),
    "mx_comm_create_rccl": (C.c_int, [C.c_int, C.c_int, C.c_int, P, C.c_size_t, C.POINTER(P)]),
    "mx_comm_create_self": (C.c_int, [C.c_int, C.POINTER(P)]),
    "mx_comm_create_shm": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int64, C.POINTER(P)]),
    "mx_comm_abort": (C.c_int, [P]),
    "mx_world_create_local": (C.c_int, [C.c_int, C.POINTER(P)]),
    "mx_comm_create_local": (C.c_int, [P, C.c_int, C.c_int, C.POINTER(P)]),
    "mx_world_destroy": (C.c_int, [P]),
    "mx_world_abort": (C.c_int, [P]),
    "mx_comm_destroy": (C.c_int, [P]),
    "mx_comm_info": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "mx_comm_stream": (C.c_int, [P, C.POINTER(P)]),
    "mx_comm_barrier": (C.c_int, [P]),
    "mx_layout_split": (C.c_int, [I64, C.c_int, I64P]),
    "mx_mat_create_csr": (C.c_int, [P, I64, I64, I64, I64, P, C.c_int, P, C.c_int, P, I64, C.c_int, C.c_int, C.POINTER(P)]),
    "mx_mat_create_coo": (C.c_int, [P, I64, I64, I64, I64, P, P, P, I64, C.c_int, C.c_int, C.POINTER(P)]),
    "mx_mat_create_stencil": (C.c_int, [P, C.c_int, I64, I64, I64, C.POINTER(P)]),
    "mx_mat_get_info": (C.c_int, [P, C.POINTER(MatInfo)]),
    "mx_mat_get_csr": (C.c_int, [P, P, P, P]),
    "mx_mat_get_split": (C.c_int, [P, P, P, P, P, P, P, P]),
    "mx_mat_mult": (C.c_int, [P, P, P]),
    "mx_mat_get_diagonal": (C.c_int, [P, P]),
    "mx_mat_bench_mult": (C.c_int, [P, P, P, C.c_int, DP, DP]),
    "mx_mat_bench_mult_cold": (C.c_int, [P, P, P, P, I64, C.c_int, DP, DP]),
    "mx_mat_destroy": (C.c_int, [P]),
    "mx_vec_dot": (C.c_int, [P, I64, P, P, DP]),
    "mx_vec_norm2": (C.c_int, [P, I64, P, DP]),
    "mx_vec_axpy": (C.c_int, [P, I64, C.c_double, P, P]),
    "mx_vec_aypx": (C.c_int, [P, I64, C.c_double, P, P]),
    "mx_vec_pointwise_mult": (C.c_int, [P, I64, P, P, P]),
    "mx_vec_scale": (C.c_int, [P, I64, C.c_double, P]),
    "mx_vec_set": (C.c_int, [P, I64, C.c_double, P]),
    "mx_vec_rhs_hash": (C.c_int, [P, I64, I64, P]),
    "mx_vec_mdot": (C.c_int, [P, I64, P, C.c_int, C.POINTER(P), DP]),
    "mx_vec_maxpy": (C.c_int, [P, I64, P, C.c_int, DP, C.POINTER(P)]),
    "mx_ksp_destroy": (C.c_int, [P]),
    "mx_finalize": (C.c_int, []),
    "mx_ksp_solve": (C.c_int, [P, C.POINTER(KSPParams), P, P, C.POINTER(KSPResult), P]),
    "mx_ksp_default_params": (None, [C.POINTER(KSPParams)]),
    "mx_lu_solve_csr": (C.c_int, [P, I64, P, P, P, P, P]),
    "mx_debug_set": (C.c_int, [C.c_int, C.c_int]),
    "mx_debug_dispatch_counts": (C.c_int, [C.POINTER(C.c_int64), C.c_int, C.c_int]),
    "mx_debug_assembly_times": (C.c_int, [C.POINTER(C.c_double), C.c_int]),
    "mx_debug_stream_read": (C.c_int, [P, P, I64, C.c_int, P]),
    "mx_debug_comm_bench": (C.c_int, [P, P, C.c_int, C.c_int, DP]),
    "mx_debug_comm_stall": (C.c_int, [P, C.c_int]),
    "mx_dev_alloc": (C.c_int, [C.c_int, C.c_size_t, C.POINTER(P)]),
    "mx_dev_free": (C.c_int, [P]),
}

_lib = None


def load():
    """Load libmxsolve.so once; raise (never fall back) if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libmxsolve.so not built at {LIB_PATH}: run `make -C mpi-petsc4py-example_amd/csrc` "
                          "or __graft_entry__.build()")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)   # AttributeError if the ABI lost a symbol
        fn.restype = res
        fn.argtypes = args
    if lib.mx_version() != 3:
        raise ImportError("libmxsolve ABI version mismatch")
    # diagnostics / A/B runs: MXSOLVE_KNOBS="27=0+3=8192" (mx_debug_set keys, include/mxsolve.h)
    for kv in filter(None, os.environ.get("MXSOLVE_KNOBS", "").split("+")):
        k, v = kv.split("=")
        lib.mx_debug_set(int(k), int(v))
    _lib = lib
    return lib


def last_error() -> str:
    buf = C.create_string_buffer(2048)
    load().mx_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc: int):
    if rc != MX_OK:
        raise MxError(rc, last_error())
    return rc


def call(name: str, *args):
    return check(getattr(load(), name)(*args))
