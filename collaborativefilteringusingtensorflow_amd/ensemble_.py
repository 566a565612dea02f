"""Ensemble drop-in, W-negative variant (src/models/pl/models/ensemble_.py):
the attention-weighted ensemble rating of the positive against each of W
negatives per pair (ensemble_.py:75-118), trained on sampler_ranking batches
with dense Adagrad on U, V, H.  Runs cf_ens_step_w (csrc/cf_ensemble.hip)."""
from .ensemble import EnsembleW


class Ensemble(EnsembleW):
    def __init__(self, n_users, n_items, kensemble=2, topN=5, split_method='cv',
                 eval_metrics=['pre', 'recall', 'mrr', 'ndcg'], reg=0.1, n_factors=20,
                 batch_size=100, max_iter=50, lr=0.1, init_mean=0.0, init_stddev=0.1,
                 device='CPU', seed=None, verbose=True):
        super(Ensemble, self).__init__(n_users, n_items, kensemble, topN, split_method,
                                       eval_metrics, reg, n_factors, batch_size, max_iter, lr,
                                       init_mean, init_stddev, device, seed, verbose)
