"""Shared train / recommend / eval loop of the four pairwise-ranking models.

Mirrors the reference's ``Model.train(fold, trasR, tstsR, sampler)``
(bprmf.py:113-170, gbprmf.py:131-183, cml.py:155-212, amf.py:187-245):

* test users = ``list(set(tstsR.nonzero()[0]))`` and their truth sets
  (bprmf.py:117-123), train items excluded from recommendations
  (bprmf.py:125, 95-103);
* ``n_batches = int(nnz / batch_size)`` steps per epoch (bprmf.py:138);
* per epoch: mean of the per-batch pre-update losses, a recommend pass,
  evaluateCV / evaluateLOOV, one log line, ``lr *= .98`` (cosmetic: the
  optimizer's lr was frozen when the train op was built).

The arithmetic runs in the native engine.  Two feeding modes:
* a device sampler from this package (sampler_ranking / sampler_uij_ranking /
  sampler_gbpr): fused on-device sample + step loop (cf_train_steps);
* any other object with ``next_batch()`` (e.g. the reference's own thread
  sampler): host-fed steps (cf_step) on exactly the batches it yields.
"""
import sys

import numpy as np

from . import _native as N
from .engine import Engine
from .io_util import to_csr
from .ranking import evaluateCV, evaluateLOOV


def parse_device(device):
    """The reference picks a TF device type ('CPU'/'GPU', bprmf.py:27); the
    native engine always runs on a HIP device, so 'CPU', 'GPU', 'GPU:k',
    'cuda:k' or an int select ordinal 0 or k."""
    if isinstance(device, int):
        return device
    s = str(device)
    if ":" in s:
        return int(s.split(":")[-1])
    return 0


class PairwiseModel(object):
    MODEL = None
    TRUNCATED_INIT = True

    def __init__(self, n_users, n_items, topN, split_method, eval_metrics, n_factors,
                 batch_size, max_iter, lr, init_mean, init_stddev, device, seed=None,
                 verbose=True):
        self._n_users, self._n_items, self._topN = int(n_users), int(n_items), int(topN)
        self._split_method, self._eval_metrics = split_method, list(eval_metrics)
        self._n_factors, self._batch_size = int(n_factors), int(batch_size)
        self._max_iter, self._lr = int(max_iter), float(lr)
        self._init_mean, self._init_stddev = float(init_mean), float(init_stddev)
        self._device = parse_device(device)
        self._seed = seed
        self._verbose = verbose
        self._engine = None
        self._train_lr = float(lr)  # the value the optimizer is built with
        self._init_tables = None

    # ---- hooks ----------------------------------------------------------------
    def _engine_kwargs(self):
        return {}

    def _log_line(self, fold, it, aveloss, scores, timecost):
        return ("%s_fold=%d iter=%2d: " % (self._split_method, fold, it + 1)
                + "TraLoss=%.4f lr=%.4f" % (aveloss, self._lr) + "\tTst@" + str(self._topN) + ":"
                + " ".join(m + "=%.4f" % s for m, s in zip(self._eval_metrics, scores)))

    def _after_epoch(self, it):
        pass

    def _after_train(self, fold, test_users, yss_true, scores):
        return scores

    # ---- pieces -----------------------------------------------------------------
    def _make_engine(self, n_neg, gsize, seed):
        e = Engine(self.MODEL, self._n_users, self._n_items, self._n_factors, n_neg=n_neg,
                   gsize=max(gsize, 1), lr=self._train_lr, device=self._device, seed=seed,
                   **self._engine_kwargs())
        return e

    def _recommend(self, test_users, topN=None):
        k = self._topN if topN is None else topN
        idx = self._engine.score_topk(np.asarray(test_users, dtype=np.int32), k,
                                      exclude_train=True)
        return [[int(x) for x in row if x >= 0] for row in idx]

    def _eval(self, yss_true, yss_pred):
        if self._split_method == "cv":
            return evaluateCV(yss_true, yss_pred, self._eval_metrics, self._topN)
        if self._split_method == "loov":
            return evaluateLOOV(yss_true, yss_pred, self._eval_metrics, self._topN)
        return None

    # ---- the train loop ----------------------------------------------------------------
    def train(self, fold, trasR, tstsR, sampler):
        import time
        t_indptr, t_indices, _ = to_csr(tstsR)
        test_users = list(set(np.asarray(tstsR.nonzero()[0])))
        yss_true = None
        if self._split_method == "cv":
            yss_true = [set(t_indices[t_indptr[u]:t_indptr[u + 1]].tolist()) for u in test_users]
        elif self._split_method == "loov":
            yss_true = [int(t_indices[t_indptr[u]]) for u in test_users]
        indptr, indices, _ = to_csr(trasR)
        nnz = int(indices.shape[0])
        n_batches = int(nnz / self._batch_size)

        device_fed = bool(getattr(sampler, "_cf_device_sampler", False))
        first = None
        if device_fed:
            n_neg, gsize, seed = sampler.n_neg, sampler.gsize, sampler.seed
            B = sampler.batch_size
        else:
            first = sampler.next_batch()
            if isinstance(first, np.ndarray):  # uij sampler: [B,3]
                first = (first[:, :2], first[:, 2:])
            n_neg = np.asarray(first[1]).reshape(len(first[0]), -1).shape[1]
            gsize = np.asarray(first[2]).reshape(len(first[0]), -1).shape[1] if len(first) > 2 else 0
            seed = self._seed if self._seed is not None else 1
            B = len(first[0])
        if self.MODEL == N.CF_GBPR and gsize < 1:
            raise ValueError("GBPRMF needs a sampler that yields group users")
        if self._engine is not None:
            self._engine.close()
        self._engine = self._make_engine(n_neg, gsize, seed)
        eng = self._engine
        eng.set_interactions(indptr, indices)
        init_seed = self._seed if self._seed is not None else (seed ^ 0x1234567)
        eng.init_params(self._init_mean, self._init_stddev, truncated=self.TRUNCATED_INIT,
                        seed=init_seed)
        if self._init_tables is not None:
            for name, arr in self._init_tables.items():
                eng.set_table(name, arr)
        if device_fed:
            eng.set_sampler_state(*sampler.state())

        scores = None
        for it in range(self._max_iter):
            t0 = time.time()
            if device_fed:
                aveloss = eng.train_steps(B, n_batches) / max(n_batches, 1)
            else:
                for _ in range(n_batches):
                    batch = first if first is not None else sampler.next_batch()
                    first = None
                    if isinstance(batch, np.ndarray):
                        batch = (batch[:, :2], batch[:, 2:])
                    eng.step(*batch, return_loss=False)
                aveloss = eng.take_loss() / max(n_batches, 1)
            timecost = time.time() - t0
            yss_pred = self._recommend(test_users)
            scores = self._eval(yss_true, yss_pred)
            if self._verbose:
                print(self._log_line(fold, it, aveloss, scores, timecost))
                sys.stdout.flush()
            self._lr *= .98
            self._after_epoch(it)
        if device_fed:
            sampler.set_state(*eng.sampler_state())
        return self._after_train(fold, test_users, yss_true, scores)

    def close(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None

    # ---- extras (not in the reference; used by tests and the bench) ----------------------
    @property
    def engine(self):
        return self._engine

    def set_initial_tables(self, user=None, item=None, bias=None):
        """Start the next ``train`` from these tables instead of the seeded
        initializer (the reference's TF initializers are unseeded)."""
        t = {}
        for name, arr in (("user", user), ("item", item), ("bias", bias)):
            if arr is not None:
                t[name] = np.asarray(arr, dtype=np.float32)
        self._init_tables = t or None
