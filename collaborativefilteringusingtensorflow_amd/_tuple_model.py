"""Train loop of the tuple ranking models (PRIGP, CPLR): the reference's
``train(fold, trasR, tstsR)`` (prigp.py:172-228, cplr_u.py:179-291) --
similarity and coefficient preprocessing, its own sampler, ``n_batches =
int(nnz / batch_size)`` host-fed engine steps per epoch (cf_step_plr), then
recommend + evaluate like the pairwise models."""
import sys
import time

import numpy as np

from . import _native as N
from ._model import PairwiseModel
from .io_util import to_csr


class TupleModel(PairwiseModel):
    MODEL = N.CF_PLR
    PLR_KIND = 0
    TRUNCATED_INIT = True

    def _prepare(self, trasR):
        """-> (sampler, print line); sets nothing on the engine."""
        raise NotImplementedError

    def _make_engine(self, n_neg, gsize, seed):
        from .engine import Engine
        return Engine(self.MODEL, self._n_users, self._n_items, self._n_factors, lr=self._train_lr,
                      device=self._device, seed=seed, plr_kind=self.PLR_KIND,
                      **self._engine_kwargs())

    def _next(self, sampler):
        b = sampler.next_batch()
        return (b, None) if isinstance(b, np.ndarray) else b

    def train(self, fold, trasR, tstsR, sampler=None):
        t_indptr, t_indices, _ = to_csr(tstsR)
        test_users = list(set(np.asarray(tstsR.nonzero()[0])))
        yss_true = None
        if self._split_method == "cv":
            yss_true = [set(t_indices[t_indptr[u]:t_indptr[u + 1]].tolist()) for u in test_users]
        elif self._split_method == "loov":
            yss_true = [int(t_indices[t_indptr[u]]) for u in test_users]
        indptr, indices, _ = to_csr(trasR)
        n_batches = int(indices.shape[0] / self._batch_size)
        if sampler is None:
            sampler = self._prepare(trasR)
        seed = self._seed if self._seed is not None else 1
        if self._engine is not None:
            self._engine.close()
        self._engine = self._make_engine(0, 0, seed)
        eng = self._engine
        eng.set_interactions(indptr, indices)
        eng.init_params(self._init_mean, self._init_stddev, truncated=self.TRUNCATED_INIT,
                        seed=seed ^ 0x1234567)
        if self._init_tables is not None:
            for name, arr in self._init_tables.items():
                eng.set_table(name, arr)
        scores = None
        for it in range(self._max_iter):
            t0 = time.time()
            for _ in range(n_batches):
                tuples, coefs = self._next(sampler)
                eng.step_plr(tuples, coefs, return_loss=False)
            aveloss = eng.take_loss() / max(n_batches, 1)
            timecost = time.time() - t0
            scores = self._eval(yss_true, self._recommend(test_users))
            if self._verbose:
                print(self._log_line(fold, it, aveloss, scores, timecost)
                      + "\t\ttimecost=%d(s)" % int(timecost))
                sys.stdout.flush()
            self._lr *= .98
        return scores
