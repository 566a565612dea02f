"""Ensemble drop-in, mixed variant (src/models/pl/models/ensemble__.py): every
member's own BPR loss plus ensemble_lambda times the W-negative ensemble loss
(ensemble__.py:102-145), reg on the looked-up rows and H, dense Adagrad on
U, V, H; sampler_ranking batches.  Runs cf_ens_step_w with singles on."""
from .ensemble import EnsembleW


class Ensemble(EnsembleW):
    LAM_FROM_ARG = True
    SINGLES = True

    def __init__(self, n_users, n_items, kensemble=2, ensemble_lambda=0.1, topN=5,
                 split_method='cv', eval_metrics=['pre', 'recall', 'mrr', 'ndcg'], reg=0.1,
                 n_factors=20, batch_size=100, max_iter=50, lr=0.1, init_mean=0.0,
                 init_stddev=0.1, device='CPU', seed=None, verbose=True):
        super(Ensemble, self).__init__(n_users, n_items, kensemble, topN, split_method,
                                       eval_metrics, reg, n_factors, batch_size, max_iter, lr,
                                       init_mean, init_stddev, device, seed, verbose)
        self.ensemble_lambda = float(ensemble_lambda)
