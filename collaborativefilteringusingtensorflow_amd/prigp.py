"""PRIGP drop-in (src/models/pl/models/prigp.py:17-231).

Tuples (u, i, j, t, k) from the user's top-K neighbours' items
(sampler_prigp.py); loss sum -log s(ui - uj) + alpha * sum -log s(ut - uk)
with s_x = <U_u, V_x> + b_x, + reg (l2(U_u) + l2(V_items) + l2(b_items))
(prigp.py:99-130); Adagrad on U and V only -- the item bias stays at its
initial value (var_list, prigp.py:145).  Predict U.V^T + b (prigp.py:136-139).
Run by the engine's tuple kernel (CF_PLR, cf_step_plr)."""
from . import _native as N
from ._tuple import PRIGPSampler, coefficients, top_k_rows, user_similarity
from ._tuple_model import TupleModel


class PRIGP(TupleModel):
    PLR_KIND = N.CF_PLR_PRIGP

    def __init__(self, n_users, n_items, topK=50, topN=5, split_method='cv',
                 eval_metrics=['pre', 'recall', 'map', 'mrr', 'ndcg'], alpha=1., reg=0.01,
                 n_factors=20, batch_size=1000, max_iter=50, lr=0.1, init_mean=0.0,
                 init_stddev=0.1, device='GPU', seed=None, verbose=True):
        super(PRIGP, self).__init__(n_users, n_items, topN, split_method, eval_metrics, n_factors,
                                    batch_size, max_iter, lr, init_mean, init_stddev, device, seed,
                                    verbose)
        self._topK, self._alpha, self._reg = int(topK), float(alpha), float(reg)

    def _engine_kwargs(self):
        return dict(reg=self._reg, alpha=self._alpha)

    def _prepare(self, trasR):
        simMat = top_k_rows(user_similarity(trasR), self._topK)         # prigp.py:174
        self.coefMat = coefficients(simMat, trasR, weighted=False)      # prigp.py:175
        return PRIGPSampler(trasR, self.coefMat, self._batch_size, seed=self._seed)
