"""CML driver (src/models/pl/testcml.py:18-102): same globals and worker."""
import os

from ..cml import CML
from ..sampler_ranking import Sampler
from ._common import args, load_fold, run_folds

folds = 5
binarize_threshold = 3
topN = 10
split_method = 'cv'
eval_metrics = ['pre', 'recall', 'map', 'mrr', 'ndcg']
margin = 1.
reg_cov = 1.
use_rank_weight = True
clip_norm = 1.0
n_factors = 50
batch_size = 50
negSample = 5


def worker(fold, n_users, n_items, dataset_dir):
    trasR, tstsR = load_fold(dataset_dir, fold, n_users, n_items, binarize_threshold)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1), trasR.shape, trasR.nnz,
          '%.2f' % (trasR.nnz / float(trasR.shape[0])))
    sampler = Sampler(trasR, n_neg=negSample, batch_size=batch_size)
    cml = CML(n_users, n_items, topN, split_method, eval_metrics, reg_cov, margin,
              use_rank_weight, clip_norm, n_factors, batch_size,
              device=int(os.environ.get("CF_DEVICE", "0")))
    scores = cml.train(fold + 1, trasR, tstsR, sampler)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1),
          ','.join(['%s' % m for m in eval_metrics]) + '@%d=' % topN +
          ','.join(['%.6f' % s for s in scores]))
    cml.close()
    sampler.close()
    return scores


if __name__ == '__main__':
    dataset_dir, nfolds, parallel = args(2)
    run_folds(worker, 943, 1682, dataset_dir, nfolds, 1000, eval_metrics, parallel)
