"""CML drop-in (src/models/pl/models/cml.py:12-214).

Constructor order of cml.py:14-20.  Per batch (cml.py:55-109):
    dp = |U_u-V_i|^2, dn_w = |U_u-V_jw|^2, hinge relu(dp - min_w dn_w + margin)
    weighted by log(1 + n_items * mean_w[dp - dn_w + margin > 0]),
    + reg_cov*(l2(U_u)+l2(V_i)+l2(V_negs)) when reg_cov > 0,
Adagrad, then every row of U and V clipped to L2 norm <= clip_norm
(cml.py:119-129; the engine clips all rows once after the first step and the
touched rows after every step -- untouched rows are fixed points).
Predict = -|U_u - V_i|^2 (cml.py:111-117).  Initialised with random_normal
(cml.py:32-37).  After the last epoch it evaluates topN in
{5,10,20,50,100,200,500,1000} from one top-1000 list and returns the
topN=1000 scores (cml.py:203-212).
"""
from . import _native as N
from ._model import PairwiseModel


class CML(PairwiseModel):
    MODEL = N.CF_CML
    TRUNCATED_INIT = False

    def __init__(self, n_users, n_items, topN=5, split_method='cv',
                 eval_metrics=['pre', 'recall', 'mrr', 'ndcg'], reg_cov=1., margin=1.5,
                 use_rank_weight=True, clip_norm=1.0, n_factors=20, batch_size=100,
                 max_iter=50, lr=0.1, init_mean=0.0, init_stddev=0.1, device='GPU', seed=None,
                 verbose=True):
        super(CML, self).__init__(n_users, n_items, topN, split_method, eval_metrics,
                                  n_factors, batch_size, max_iter, lr, init_mean, init_stddev,
                                  device, seed, verbose)
        self._reg_cov, self._margin = float(reg_cov), float(margin)
        self._use_rank_weight, self._clip_norm = bool(use_rank_weight), float(clip_norm)

    def _engine_kwargs(self):
        return dict(reg_cov=self._reg_cov, margin=self._margin,
                    use_rank_weight=self._use_rank_weight, clip_norm=self._clip_norm)

    def _after_train(self, fold, test_users, yss_true, scores):
        topNs = [5, 10, 20, 50, 100, 200, 500, 1000]
        self._topN = topNs[-1]
        yss_pred = self._recommend(test_users)
        for topN in topNs:
            self._topN = topN
            scores = self._eval(yss_true, yss_pred)
            if self._verbose:
                print("%s_fold=%d: " % (self._split_method, fold),
                      '\tTst@' + str(self._topN) + ':' + ' '.join(
                          m + '=%.4f' % s for m, s in zip(self._eval_metrics, scores)))
        return scores
