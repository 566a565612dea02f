"""Ensemble drop-in (src/models/pl/models/ensemble.py:12-232): K attention-
weighted MF members trained on ``sampler_uij_ranking`` (u, i, j) batches.

The arithmetic -- the reference graph's [B, B] pairwise loss (its [B] x [B, 1]
broadcast, ensemble.py:84-91), the softmax over members, dense Adagrad on U,
V, H (ensemble.py:146) -- runs in the native ensemble object
(csrc/cf_ensemble.hip, ``cf_ens_*``); this module is the host loop.

``Ensemble.train(fold, trasR, tstsR, sampler)`` follows ensemble.py:173-229:
test users / truth sets / train-item filter as in the pairwise models,
``n_batches = int(nnz / batch_size)`` host-fed steps per epoch, the mean
pre-update batch loss, a recommend + evaluate pass and the log line.  The
``lr *= .98`` there is cosmetic: the optimizer was built with the initial lr
(ensemble.py:146 at line 194), as in every other model.
"""
import ctypes
import sys
import time

import numpy as np

from . import _native as N
from ._model import parse_device
from .io_util import to_csr
from .ranking import evaluateCV, evaluateLOOV

TABLES = {"user": 0, "item": 1, "h": 2, "acc_user": 3, "acc_item": 4, "acc_h": 5}


def _ptr(a, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


class EnsembleEngine(object):
    """One HIP device's ensemble tables U [K, n_users, d], V [K, n_items, d],
    H [K, d] and their Adagrad accumulators."""

    def __init__(self, n_users, n_items, kensemble, n_factors, reg=0.1, lr=0.1, acc_init=0.1,
                 device=0):
        L = N.lib()
        self._L = L
        self.n_users, self.n_items = int(n_users), int(n_items)
        self.K, self.d = int(kensemble), int(n_factors)
        self._h = ctypes.c_void_p()
        N.check(L.cf_ens_create(self.n_users, self.n_items, self.K, self.d, float(reg), float(lr),
                                float(acc_init), int(device), ctypes.byref(self._h)),
                "cf_ens_create")

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._L.cf_ens_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _shape(self, name):
        t = TABLES[name] % 3
        return ((self.K, self.n_users, self.d), (self.K, self.n_items, self.d), (self.K, self.d))[t]

    def init_params(self, mean=0.0, stddev=0.1, truncated=True, seed=1):
        N.check(self._L.cf_ens_init_params(self._h, float(mean), float(stddev), int(bool(truncated)),
                                           int(seed) & 0xFFFFFFFFFFFFFFFF), "cf_ens_init_params")

    def set_lr(self, lr):
        N.check(self._L.cf_ens_set_lr(self._h, float(lr)), "cf_ens_set_lr")

    def set_table(self, name, arr):
        a = np.ascontiguousarray(arr, dtype=np.float32)
        if a.shape != self._shape(name):
            raise ValueError("%s must be %s, got %s" % (name, self._shape(name), a.shape))
        N.check(self._L.cf_ens_set_table(self._h, TABLES[name], _ptr(a, ctypes.c_float), a.size),
                "cf_ens_set_table")

    def get_table(self, name):
        a = np.empty(self._shape(name), dtype=np.float32)
        N.check(self._L.cf_ens_get_table(self._h, TABLES[name], _ptr(a, ctypes.c_float), a.size),
                "cf_ens_get_table")
        return a

    def set_interactions(self, indptr, indices):
        ip = np.ascontiguousarray(indptr, dtype=np.int64)
        ix = np.ascontiguousarray(indices, dtype=np.int32)
        N.check(self._L.cf_ens_set_interactions(self._h, _ptr(ip, ctypes.c_int64),
                                                _ptr(ix, ctypes.c_int32), ix.shape[0]),
                "cf_ens_set_interactions")

    def step(self, uij, return_loss=True):
        t = np.ascontiguousarray(uij, dtype=np.int32)
        if t.ndim != 2 or t.shape[1] != 3:
            raise ValueError("uij must be [B, 3]")
        loss = ctypes.c_double(0.0)
        N.check(self._L.cf_ens_step(self._h, _ptr(t, ctypes.c_int32), t.shape[0],
                                    ctypes.byref(loss) if return_loss else None), "cf_ens_step")
        return float(loss.value) if return_loss else None

    def step_w(self, pairs, negs, lam=1.0, singles=False, return_loss=True):
        """One step of the W-negative variants (cf_ens_step_w): pairs [B, 2],
        negs [B, W]."""
        pr = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
        B = pr.shape[0]
        ng = np.ascontiguousarray(negs, dtype=np.int32).reshape(B, -1)
        loss = ctypes.c_double(0.0)
        N.check(self._L.cf_ens_step_w(self._h, _ptr(pr, ctypes.c_int32), _ptr(ng, ctypes.c_int32),
                                      ng.shape[1], B, float(lam), 1 if singles else 0,
                                      ctypes.byref(loss) if return_loss else None), "cf_ens_step_w")
        return float(loss.value) if return_loss else None

    def take_loss(self):
        s = ctypes.c_double(0.0)
        N.check(self._L.cf_ens_take_loss(self._h, ctypes.byref(s)), "cf_ens_take_loss")
        return float(s.value)

    def score_topk(self, users, k, exclude_train=True, return_values=False):
        u = np.ascontiguousarray(users, dtype=np.int32)
        idx = np.empty((u.shape[0], int(k)), dtype=np.int32)
        val = np.empty((u.shape[0], int(k)), dtype=np.float32) if return_values else None
        N.check(self._L.cf_ens_score_topk(self._h, _ptr(u, ctypes.c_int32), u.shape[0], int(k),
                                          int(bool(exclude_train)), _ptr(idx, ctypes.c_int32),
                                          _ptr(val, ctypes.c_float) if val is not None else None),
                "cf_ens_score_topk")
        return (idx, val) if return_values else idx


class Ensemble(object):
    def __init__(self, n_users, n_items, kensemble=3, topN=5, split_method='cv',
                 eval_metrics=['pre', 'recall', 'mrr', 'ndcg'], reg=0.1, n_factors=20,
                 batch_size=100, max_iter=50, lr=0.1, init_mean=0.0, init_stddev=0.1,
                 device='CPU', seed=None, verbose=True):
        self._n_users, self._n_items, self._topN = int(n_users), int(n_items), int(topN)
        self._split_method, self._eval_metrics = split_method, list(eval_metrics)
        self._reg, self._n_factors, self._batch_size = float(reg), int(n_factors), int(batch_size)
        self._max_iter, self._lr = int(max_iter), float(lr)
        self._train_lr = float(lr)
        self._init_mean, self._init_stddev = float(init_mean), float(init_stddev)
        self._device = parse_device(device)
        self.kensemble = int(kensemble)
        self._seed = seed
        self._verbose = verbose
        self._engine = None
        self._init_tables = None

    @property
    def engine(self):
        return self._engine

    def set_initial_tables(self, user=None, item=None, h=None):
        """Start the next ``train`` from these tables instead of the seeded
        truncated-normal initializer (the reference's is unseeded)."""
        t = {n: np.asarray(a, dtype=np.float32) for n, a in (("user", user), ("item", item), ("h", h))
             if a is not None}
        self._init_tables = t or None

    def _feed(self, eng, batch):
        eng.step(batch, return_loss=False)   # [B, 3] (u, i, j), ensemble.py:204-205

    def _recommend(self, test_users):
        idx = self._engine.score_topk(np.asarray(test_users, dtype=np.int32), self._topN,
                                      exclude_train=True)
        return [[int(x) for x in row if x >= 0] for row in idx]

    def _eval(self, yss_true, yss_pred):
        if self._split_method == 'cv':
            return evaluateCV(yss_true, yss_pred, self._eval_metrics, self._topN)
        if self._split_method == 'loov':
            return evaluateLOOV(yss_true, yss_pred, self._eval_metrics, self._topN)
        return None

    def train(self, fold, trasR, tstsR, sampler):
        t_indptr, t_indices, _ = to_csr(tstsR)
        test_users = list(set(np.asarray(tstsR.nonzero()[0])))
        yss_true = None
        if self._split_method == 'cv':
            yss_true = [set(t_indices[t_indptr[u]:t_indptr[u + 1]].tolist()) for u in test_users]
        elif self._split_method == 'loov':
            yss_true = [int(t_indices[t_indptr[u]]) for u in test_users]
        indptr, indices, _ = to_csr(trasR)
        n_batches = int(indices.shape[0] / self._batch_size)
        if self._engine is not None:
            self._engine.close()
        self._engine = eng = EnsembleEngine(self._n_users, self._n_items, self.kensemble,
                                            self._n_factors, reg=self._reg, lr=self._train_lr,
                                            device=self._device)
        eng.set_interactions(indptr, indices)
        seed = self._seed if self._seed is not None else 1
        eng.init_params(self._init_mean, self._init_stddev, truncated=True, seed=seed ^ 0x1234567)
        if self._init_tables is not None:
            for name, arr in self._init_tables.items():
                eng.set_table(name, arr)
        scores = None
        for it in range(self._max_iter):
            t0 = time.time()
            for _ in range(n_batches):
                self._feed(eng, sampler.next_batch())
            aveloss = eng.take_loss() / max(n_batches, 1)
            scores = self._eval(yss_true, self._recommend(test_users))
            if self._verbose:
                print("%s_fold=%d iter=%2d: " % (self._split_method, fold, it + 1),
                      "TraLoss=%.4f lr=%.4f" % (aveloss, self._lr),
                      '\tTst@' + str(self._topN) + ':' + ' '.join(
                          [m + '=%.4f' % s for m, s in zip(self._eval_metrics, scores)]),
                      "\ttimecost=%.1f(s)" % (time.time() - t0))
                sys.stdout.flush()
            self._lr *= .98
        return scores

    def close(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None


class EnsembleW(Ensemble):
    """Shared host loop of the W-negative variants (ensemble_.py,
    ensemble__.py): sampler_ranking batches (pairs [B, 2], negs [B, W]),
    cf_ens_step_w with the variant's lam / singles."""
    LAM_FROM_ARG = False
    SINGLES = False

    def _feed(self, eng, batch):
        pairs, negs = batch
        lam = self.ensemble_lambda if self.LAM_FROM_ARG else 1.0
        eng.step_w(pairs, negs, lam=lam, singles=self.SINGLES, return_loss=False)
