"""GBPRMF drop-in (src/models/pl/models/gbprmf.py:13-186).

Constructor order of gbprmf.py:14-19.  Per batch (gbprmf.py:58-89):
    ui = rho*mean_k<U_gk,V_i> + (1-rho)<U_u,V_i> + b_i,  uj = <U_u,V_j> + b_j
    loss = sum(-log sigmoid(ui-uj)) + reg*(l2(U_u)+l2(U_g)+l2(V_i)+l2(b_negs))
(no L2 on V_negs or b_i -- kept for parity), Adagrad over U, V, b.
Predict = U.V^T + b (gbprmf.py:95-99).  Log lines carry a timestamp and the
epoch wall time like gbprmf.py:174-179.
"""
import datetime as dt

from . import _native as N
from ._model import PairwiseModel


class GBPRMF(PairwiseModel):
    MODEL = N.CF_GBPR

    def __init__(self, n_users, n_items, topN=10, rho=.5, gsize=2, split_method='cv',
                 eval_metrics=['pre', 'recall', 'mrr', 'ndcg'], reg=0.02, n_factors=20,
                 batch_size=100, max_iter=30, lr=0.1, init_mean=0.0, init_stddev=0.1,
                 device='GPU', seed=None, verbose=True):
        super(GBPRMF, self).__init__(n_users, n_items, topN, split_method, eval_metrics,
                                     n_factors, batch_size, max_iter, lr, init_mean, init_stddev,
                                     device, seed, verbose)
        self._rho, self._gsize, self._reg = float(rho), int(gsize), float(reg)

    def _engine_kwargs(self):
        return dict(reg=self._reg, rho=self._rho)

    def _log_line(self, fold, it, aveloss, scores, timecost):
        return (dt.datetime.now().strftime('%m-%d %H:%M:%S') + " "
                + "%s_fold=%d iter=%2d: " % (self._split_method, fold, it + 1)
                + "TraLoss=%.4f lr=%.4f" % (aveloss, self._lr) + "\tTst@" + str(self._topN) + ":"
                + " ".join(m + "=%.4f" % s for m, s in zip(self._eval_metrics, scores))
                + "\t\ttimecost=%d(s)" % int(timecost))
