"""Rating-file ingest: drop-in for ``src/utils/IOUtil.py`` and ``src/utils/Util.py``.

Same names and rules:
* ``split_row``: split on ',' if present, else ';', else whitespace (Util.py:5-11);
* ``loadSparseR``: 2-field lines set 1, 3-field lines set float(rating), any
  other field count is ignored; a later line overwrites an earlier one
  (IOUtil.py:23-32);
* ``matBinarize``: ``(R > threshold)`` as float32 (Util.py:15-16).

Plus ``to_csr``: the sorted, duplicate-free CSR the engine consumes (the
nnz order of ``trasR.nonzero()``, sampler_ranking.py:13).
"""
import numpy as np
import scipy.sparse as sp

__all__ = ["split_row", "loadSparseR", "saveTriads", "matBinarize", "to_csr"]


def split_row(row_content):
    s = row_content.strip()
    for sep in (",", ";"):
        if sep in row_content:
            return s.split(sep)
    return s.split()


def loadSparseR(usernum, itemnum, inFilePath):
    entries = {}
    with open(inFilePath, "r") as f:
        for line in f:
            fields = split_row(line)
            if len(fields) == 2:
                entries[(int(fields[0]), int(fields[1]))] = 1.0
            elif len(fields) == 3:
                entries[(int(fields[0]), int(fields[1]))] = float(fields[2])
    R = sp.lil_matrix((usernum, itemnum))
    if entries:
        keys = np.array(list(entries.keys()), dtype=np.int64)
        vals = np.array(list(entries.values()), dtype=np.float64)
        coo = sp.coo_matrix((vals, (keys[:, 0], keys[:, 1])), shape=(usernum, itemnum))
        coo.eliminate_zeros()  # assigning 0 into a lil_matrix stores nothing
        R = sp.lil_matrix(coo)
    return R


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
