"""Rating-file ingest: drop-in for ``src/utils/IOUtil.py`` and ``src/utils/Util.py``.

Same names and rules:
* ``split_row``: split on ',' if present, else ';', else whitespace (Util.py:5-11);
* ``loadSparseR``: 2-field lines set 1, 3-field lines set float(rating), any
  other field count is ignored; a later line overwrites an earlier one
  (IOUtil.py:23-32);
* ``matBinarize``: ``(R > threshold)`` as float32 (Util.py:15-16).

Plus ``to_csr``: the sorted, duplicate-free CSR the engine consumes (the
nnz order of ``trasR.nonzero()``, sampler_ranking.py:13), and ``load_csr``:
file -> (binarised) CSR straight from the native parser (cf_ratings_load,
include/cf_engine.h), without the lil_matrix detour.

``loadSparseR`` parses with the native multi-threaded ingest
(csrc/cf_ingest.cpp) and returns the lil_matrix the reference returns.
"""
import ctypes

import numpy as np
import scipy.sparse as sp

from . import _native as N

__all__ = ["split_row", "loadSparseR", "saveTriads", "matBinarize", "to_csr", "load_csr"]


def _ratings(path, n_users, n_items, n_threads=0):
    L = N.lib()
    h = ctypes.c_void_p()
    nnz = ctypes.c_int64(0)
    N.check(L.cf_ratings_load(str(path).encode(), int(n_users), int(n_items), int(n_threads),
                              ctypes.byref(h), ctypes.byref(nnz)), "cf_ratings_load")
    return L, h


def _csr(L, h, n_users, binarize, threshold):
    nnz = ctypes.c_int64(0)
    N.check(L.cf_ratings_csr(h, 1 if binarize else 0, float(threshold), None, None, None,
                             ctypes.byref(nnz)), "cf_ratings_csr")
    indptr = np.zeros(int(n_users) + 1, dtype=np.int64)
    indices = np.zeros(nnz.value, dtype=np.int32)
    values = np.zeros(nnz.value, dtype=np.float64)
    N.check(L.cf_ratings_csr(h, 1 if binarize else 0, float(threshold),
                             indptr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                             indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                             values.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                             ctypes.byref(nnz)), "cf_ratings_csr")
    return indptr, indices, values


def load_csr(path, n_users, n_items, threshold=None, n_threads=0):
    """Rating file -> CSR (indptr int64, indices int32 sorted per row).
    With ``threshold``: matBinarize(loadSparseR(...), threshold)'s pattern;
    without: (indptr, indices, ratings float64) of loadSparseR(...)."""
    L, h = _ratings(path, n_users, n_items, n_threads)
    try:
        ip, ix, v = _csr(L, h, n_users, threshold is not None, threshold or 0.0)
    finally:
        L.cf_ratings_free(h)
    return (ip, ix) if threshold is not None else (ip, ix, v)


def split_row(row_content):
    s = row_content.strip()
    for sep in (",", ";"):
        if sep in row_content:
            return s.split(sep)
    return s.split()


def loadSparseR(usernum, itemnum, inFilePath):
    """IOUtil.py:8-16: the rating file as a (usernum x itemnum) lil_matrix."""
    ip, ix, v = load_csr(inFilePath, usernum, itemnum)
    return sp.lil_matrix(sp.csr_matrix((v, ix, ip), shape=(usernum, itemnum)))


def saveTriads(triads, outFilePath, isRatingInt=False):
    with open(outFilePath, "w") as f:
        for user, item, rating in triads:
            if isRatingInt:
                f.write("%d\t%d\t%d\n" % (int(user), int(item), rating))
            else:
                f.write("%d\t%d\t%.1f\n" % (int(user), int(item), rating))


def matBinarize(sR, r_threshold):
    return (sR > r_threshold).astype(np.float32)


def to_csr(R):
    """Binary CSR (indptr int64, indices int32, rows sorted) of any scipy
    matrix's nonzero pattern."""
    csr = sp.csr_matrix(R, dtype=np.float32)
    csr.eliminate_zeros()
    csr.sort_indices()
    csr.sum_duplicates()
    return csr.indptr.astype(np.int64), csr.indices.astype(np.int32), csr.shape
