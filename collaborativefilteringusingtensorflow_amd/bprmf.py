"""BPRMF drop-in (src/models/pl/models/bprmf.py:12-173).

Same constructor (positional order of bprmf.py:13-18), ``train`` and
``close``.  Loss per batch (bprmf.py:52-71):
    sum(-log sigmoid(<U_u,V_i> - <U_u,V_j>)) + reg*(l2(U_u)+l2(V_i)+l2(V_negs))
optimised by TF1 Adagrad (acc0 = 0.1, constant lr; bprmf.py:83-88), run by the
native gfx950 engine.  Predict = U.V^T (bprmf.py:77-81).
"""
from . import _native as N
from ._model import PairwiseModel


class BPRMF(PairwiseModel):
    MODEL = N.CF_BPR

    def __init__(self, n_users, n_items, topN=5, split_method='cv',
                 eval_metrics=['pre', 'recall', 'mrr', 'ndcg'], reg=0.02, n_factors=20,
                 batch_size=100, max_iter=50, lr=0.1, init_mean=0.0, init_stddev=0.1,
                 device='GPU', seed=None, verbose=True):
        super(BPRMF, self).__init__(n_users, n_items, topN, split_method, eval_metrics,
                                    n_factors, batch_size, max_iter, lr, init_mean, init_stddev,
                                    device, seed, verbose)
        self._reg = float(reg)

    def _engine_kwargs(self):
        return dict(reg=self._reg)
