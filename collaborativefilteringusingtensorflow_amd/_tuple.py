"""Host side of the tuple ranking models (PRIGP, CPLR): the user-similarity
preprocessing and the tuple samplers.

These run once per fold (similarity, coefficients) or feed host batches to
the engine's ``cf_step_plr``; the optimizer step itself is the gfx950 kernel.

* ``user_similarity``: cosine similarity of the users' binary rows with a
  zero diagonal (prigp.py:62-70 / cplr_u.py:66-74 ``__calsim__``), vectorised.
* ``top_k_rows``: keep each row's top-K similarities (prigp.py:72-78 uses the
  last K of ``np.argsort`` unconditionally; cplr_u.py:76-87 keeps the row's
  nonzeros when it has at most K) -- the same ``np.argsort`` call, so ties
  resolve as in the reference.
* ``coefficients``: PRIGP counts, per user and item, the top-K neighbours who
  consumed the item (prigp.py:80-87); CPLR sums their similarities
  (cplr_u.py:89-96) and the train loop divides each row by its mean over the
  stored entries (cplr_u.py:194-197).
* ``PRIGPSampler`` / ``UITJSampler``: the producer loops of
  src/samplers/sampler_prigp.py:24-52 and sampler_uitj_ranking.py:22-38 on a
  seedable RandomState, without the thread and queue -- run natively
  (``cf_tuple_sampler_*``, csrc/cf_mt_sampler.cpp) on the same legacy MT19937
  stream; ``native=False`` keeps the Python loops (same batches, ~20x slower).
"""
import ctypes
import os

import numpy as np
import scipy.sparse as sp


def user_similarity(R):
    """Dense [n_users, n_users] cosine similarity, zero diagonal.  The
    reference divides row a, then column a, for a = 0, 1, ..: entry (a, b)
    is (dot / den_a) / den_b above the diagonal and (dot / den_b) / den_a
    below it.  The train matrix is float32 (matBinarize, Util.py:16), so the
    reference's similarities are float32 too.  Both are kept, so that the
    values -- and the argsort ties of the top-K step -- are the reference's."""
    B = sp.csr_matrix(R, dtype=np.float32)
    D = (B @ B.T).toarray().astype(np.float32)
    den = np.sqrt(np.asarray(B.multiply(B).sum(axis=1), dtype=np.float32).ravel())
    den = np.where(den > 0, den, np.float32(1.0)).astype(np.float32)
    upper = (D / den[:, None]) / den[None, :]
    lower = (D / den[None, :]) / den[:, None]
    S = np.where(np.triu(np.ones(D.shape, dtype=bool), 1), upper, lower)
    np.fill_diagonal(S, 0.0)
    return S


def top_k_rows(S, k, keep_short_rows=False):
    """Zero all but each row's top-k entries (in place)."""
    for r in range(S.shape[0]):
        row = S[r, :]
        if keep_short_rows and k >= np.count_nonzero(row):
            inds = row.nonzero()[0]
        else:
            inds = np.argsort(row)[-k:]
        keep = np.zeros(S.shape[1], dtype=S.dtype)
        keep[inds] = row[inds]
        S[r, :] = keep
    return S


def coefficients(S_topk, R, weighted):
    """[n_users, n_items] coefficients as a lil_matrix (zeros not stored);
    rows of users without train interactions stay empty."""
    Rb = sp.csr_matrix(R, dtype=np.float64)
    Rb.data[:] = 1.0
    W = sp.csr_matrix(S_topk if weighted else (S_topk != 0).astype(np.float64))
    C = (W @ Rb).tocsr()
    active = np.diff(Rb.indptr) > 0
    C = sp.diags(active.astype(np.float64)) @ C
    C.eliminate_zeros()
    return sp.lil_matrix(C)


def normalise_rows(C):
    """cplr_u.py:194-197: each row divided by its mean over stored entries."""
    C = sp.csr_matrix(C, dtype=np.float64)
    for r in range(C.shape[0]):
        a, b = C.indptr[r], C.indptr[r + 1]
        if b > a:
            ave = C.data[a:b].sum() / (b - a)
            if ave > 0:
                C.data[a:b] /= ave
    return sp.lil_matrix(C)


class _NativeTupleSampler(object):
    """cf_tuple_sampler over the train and coefficient CSRs."""

    def __init__(self, kind, trasR, coefMat, batch_size, seed):
        from . import _native as N
        self._N = N
        self._L = N.lib()
        self.kind, self.batch_size = int(kind), int(batch_size)
        R = sp.csr_matrix(trasR)
        R.sort_indices()
        C = sp.csr_matrix(coefMat, dtype=np.float64)
        C.sort_indices()
        self.n_users, self.n_items = R.shape
        ip = np.ascontiguousarray(R.indptr, np.int64)
        ix = np.ascontiguousarray(R.indices, np.int32)
        cp = np.ascontiguousarray(C.indptr, np.int64)
        cx = np.ascontiguousarray(C.indices, np.int32)
        cv = np.ascontiguousarray(C.data, np.float64)
        if seed is None:
            seed = int.from_bytes(os.urandom(4), "little")
        self._h = ctypes.c_void_p()
        P = ctypes.POINTER
        N.check(self._L.cf_tuple_sampler_create(
            self.kind, ip.ctypes.data_as(P(ctypes.c_int64)), ix.ctypes.data_as(P(ctypes.c_int32)),
            self.n_users, self.n_items, cp.ctypes.data_as(P(ctypes.c_int64)),
            cx.ctypes.data_as(P(ctypes.c_int32)), cv.ctypes.data_as(P(ctypes.c_double)),
            self.batch_size, int(seed) & 0xFFFFFFFF, ctypes.byref(self._h)), "cf_tuple_sampler_create")

    def _draw(self):
        B = self.batch_size
        t = np.empty((B, 5 if self.kind == 0 else 4), np.int32)
        c = np.empty((B, 2), np.float32) if self.kind == 1 else None
        self._N.check(self._L.cf_tuple_sampler_next(
            self._h, t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            c.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if c is not None else None),
            "cf_tuple_sampler_next")
        return t, c

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._L.cf_tuple_sampler_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PRIGPSampler(object):
    """sampler_prigp.py: (u, i, j, t, k) tuples; t, k drawn from the user's
    coefficient items (the more-coefficient item first)."""

    def __new__(cls, trasR, coefMat, batch_size=100, seed=None, native=True):
        if native and cls is PRIGPSampler:
            return _NativePRIGP(trasR, coefMat, batch_size, seed)
        return super(PRIGPSampler, cls).__new__(cls)

    def __init__(self, trasR, coefMat, batch_size=100, seed=None, native=False):
        self.batch_size = int(batch_size)
        self.n_users, self.n_items = trasR.shape
        self.rng = np.random.RandomState(seed)
        R = sp.lil_matrix(trasR)
        self.pairs = np.array(R.nonzero()).T
        self.pos = [set(row) for row in R.rows]
        C = sp.lil_matrix(coefMat)
        self.coef_items = [list(row) for row in C.rows]
        self.coef_sets = [set(row) for row in C.rows]
        self.coef_val = [dict(zip(row, vals)) for row, vals in zip(C.rows, C.data)]
        self.coef_nvals = [len(set(vals)) for vals in C.data]
        self.coef_nnz = [len(row) for row in C.rows]
        self._epoch_batches = 0
        self._b = 0

    def next_batch(self):
        rng, B, n_items = self.rng, self.batch_size, self.n_items
        if self._b >= self._epoch_batches:
            rng.shuffle(self.pairs)
            self._epoch_batches = len(self.pairs) // B
            self._b = 0
        batch = np.zeros((B, 5), dtype=np.int64)
        batch[:, :2] = self.pairs[self._b * B:(self._b + 1) * B]
        batch[:, 2] = rng.randint(0, n_items, size=B)
        self._b += 1
        for r in range(B):
            u, i, j = batch[r, 0], batch[r, 1], batch[r, 2]
            while j in self.pos[u]:
                batch[r, 2] = j = rng.randint(0, n_items)
            t, k = i, j
            if self.coef_nvals[u] > 0:
                items, cset, cval = self.coef_items[u], self.coef_sets[u], self.coef_val[u]
                t = items[rng.randint(len(items))]
                k = rng.randint(n_items)
                while k in cset:
                    k = rng.randint(n_items)
                if self.coef_nvals[u] > 1 and rng.randn() < self.coef_nnz[u] / float(n_items):
                    k = items[rng.randint(len(items))]
                    while cval[t] == cval[k]:
                        k = items[rng.randint(len(items))]
                    if cval[t] < cval[k]:
                        t, k = k, t
            batch[r, :] = [u, i, j, t, k]
        return batch


class _NativePRIGP(_NativeTupleSampler):
    def __init__(self, trasR, coefMat, batch_size=100, seed=None):
        super(_NativePRIGP, self).__init__(0, trasR, coefMat, batch_size, seed)

    def next_batch(self):
        return self._draw()[0].astype(np.int64)


class UITJSampler(object):
    """sampler_uitj_ranking.py: (u, i, t, j) tuples and (coef[u,i], coef[u,t])."""

    def __new__(cls, trasR, coefMat, batch_size=100, seed=None, native=True):
        if native and cls is UITJSampler:
            return _NativeUITJ(trasR, coefMat, batch_size, seed)
        return super(UITJSampler, cls).__new__(cls)

    def __init__(self, trasR, coefMat, batch_size=100, seed=None, native=False):
        self.batch_size = int(batch_size)
        self.n_users, self.n_items = trasR.shape
        self.rng = np.random.RandomState(seed)
        R = sp.lil_matrix(trasR)
        C = sp.lil_matrix(coefMat)
        self.ui = [list(row) for row in R.rows]
        self.ui_set = [set(row) for row in R.rows]
        self.ut = [sorted(set(C.rows[u]) - self.ui_set[u]) for u in range(self.n_users)]
        self.ut_set = [set(x) for x in self.ut]
        self.coef = [dict(zip(row, vals)) for row, vals in zip(C.rows, C.data)]
        self.valid = np.array([len(self.ui[u]) > 0 and len(self.ut[u]) > 0 and
                               len(self.ui[u]) + len(self.ut[u]) < self.n_items
                               for u in range(self.n_users)])
        if not self.valid.any():
            raise ValueError("no user has both train and coefficient-only items")

    def next_batch(self):
        rng, B = self.rng, self.batch_size
        out = np.zeros((B, 4), dtype=np.int64)
        coefs = np.zeros((B, 2), dtype=np.float64)
        for r in range(B):
            u = rng.randint(0, self.n_users)
            while not self.valid[u]:
                u = rng.randint(0, self.n_users)
            i = self.ui[u][rng.randint(len(self.ui[u]))]
            t = self.ut[u][rng.randint(len(self.ut[u]))]
            j = rng.randint(0, self.n_items)
            while j in self.ui_set[u] or j in self.ut_set[u]:
                j = rng.randint(0, self.n_items)
            out[r] = (u, i, t, j)
            coefs[r] = (self.coef[u].get(i, 0.0), self.coef[u].get(t, 0.0))
        return out, coefs


class _NativeUITJ(_NativeTupleSampler):
    def __init__(self, trasR, coefMat, batch_size=100, seed=None):
        super(_NativeUITJ, self).__init__(1, trasR, coefMat, batch_size, seed)

    def next_batch(self):
        t, c = self._draw()
        return t.astype(np.int64), c.astype(np.float64)
