"""CPLR drop-in (src/models/pl/models/cplr_u.py:17-294).

Tuples (u, i, t, j) with coefficients (c_ui, c_ut) from the user's top-K
neighbours (sampler_uitj_ranking.py); loss
  alpha * -log s(((c_ui+1)/(c_ut+1)) (ui - ut)) + beta * -log s((c_ut+1)(ut - uj))
  + gamma * -log s((c_ui+1)(ui - uj)) + reg (l2(U_u) + l2(V_items) + l2(b_items))
with s_x = <U_u, V_x> + b_x (cplr_u.py:106-137); Adagrad on U, V and b
(cplr_u.py:152); coefficient rows divided by their mean (cplr_u.py:194-197).
Run by the engine's tuple kernel (CF_PLR, cf_step_plr)."""
from . import _native as N
from ._tuple import UITJSampler, coefficients, normalise_rows, top_k_rows, user_similarity
from ._tuple_model import TupleModel


class CPLR(TupleModel):
    PLR_KIND = N.CF_PLR_CPLR

    def __init__(self, n_users, n_items, topK=50, topN=5, split_method='cv',
                 eval_metrics=['pre', 'recall', 'map', 'mrr', 'ndcg'], alpha=1., beta=1., gamma=1.,
                 reg=0.01, n_factors=20, batch_size=1000, max_iter=50, lr=0.1, init_mean=0.0,
                 init_stddev=0.1, device='GPU', seed=None, verbose=True):
        super(CPLR, self).__init__(n_users, n_items, topN, split_method, eval_metrics, n_factors,
                                   batch_size, max_iter, lr, init_mean, init_stddev, device, seed,
                                   verbose)
        self._topK, self._reg = int(topK), float(reg)
        self._alpha, self._beta, self._gamma = float(alpha), float(beta), float(gamma)

    def _engine_kwargs(self):
        return dict(reg=self._reg, alpha=self._alpha, beta=self._beta, gamma=self._gamma)

    def _prepare(self, trasR):
        simMat = top_k_rows(user_similarity(trasR), self._topK, keep_short_rows=True)
        self.coefMat = normalise_rows(coefficients(simMat, trasR, weighted=True))
        return UITJSampler(trasR, self.coefMat, self._batch_size, seed=self._seed)
