"""PETSc binary viewer format for Mat (AIJ) and Vec (SURVEY.md §8f row F4;
the reference's `A.view()` hook, petsc_funcs.py:8).

Layout PETSc's MatView/MatLoad and VecView/VecLoad use for binary viewers with
32-bit indices, all big-endian:
  Mat: int32 MAT_FILE_CLASSID=1211216, int32 M, int32 N, int32 nnz,
       int32 row_lengths[M], int32 cols[nnz], float64 values[nnz]
  Vec: int32 VEC_FILE_CLASSID=1211214, int32 N, float64 values[N]
Objects follow each other in one file.  Host-side I/O only; matrices are
assembled on the GPU after loading.
"""
from __future__ import annotations

import numpy as np

MAT_FILE_CLASSID = 1211216
VEC_FILE_CLASSID = 1211214


def write_mat(fh, M: int, N: int, indptr, cols, vals):
    indptr = np.asarray(indptr, dtype=np.int64)
    nnz = int(indptr[-1])
    if max(M, N, nnz) >= 2 ** 31:
        raise ValueError("32-bit PETSc binary format cannot hold this matrix")
    np.array([MAT_FILE_CLASSID, M, N, nnz], dtype=">i4").tofile(fh)
    np.diff(indptr).astype(">i4").tofile(fh)
    np.asarray(cols, dtype=np.int64).astype(">i4").tofile(fh)
    np.asarray(vals, dtype=np.float64).astype(">f8").tofile(fh)


def read_mat(fh):
    hdr = np.fromfile(fh, dtype=">i4", count=4)
    if hdr.size < 4 or hdr[0] != MAT_FILE_CLASSID:
        raise ValueError("not a PETSc binary Mat (bad class id)")
    M, N, nnz = int(hdr[1]), int(hdr[2]), int(hdr[3])
    lens = np.fromfile(fh, dtype=">i4", count=M).astype(np.int64)
    cols = np.fromfile(fh, dtype=">i4", count=nnz).astype(np.int64)
    vals = np.fromfile(fh, dtype=">f8", count=nnz).astype(np.float64)
    if lens.size != M or cols.size != nnz or vals.size != nnz or int(lens.sum()) != nnz:
        raise ValueError("truncated or inconsistent PETSc binary Mat")
    indptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return M, N, indptr, cols, vals


def write_vec(fh, vals):
    vals = np.asarray(vals, dtype=np.float64)
    np.array([VEC_FILE_CLASSID, vals.size], dtype=">i4").tofile(fh)
    vals.astype(">f8").tofile(fh)


def read_vec(fh):
    hdr = np.fromfile(fh, dtype=">i4", count=2)
    if hdr.size < 2 or hdr[0] != VEC_FILE_CLASSID:
        raise ValueError("not a PETSc binary Vec (bad class id)")
    n = int(hdr[1])
    vals = np.fromfile(fh, dtype=">f8", count=n).astype(np.float64)
    if vals.size != n:
        raise ValueError("truncated PETSc binary Vec")
    return vals
