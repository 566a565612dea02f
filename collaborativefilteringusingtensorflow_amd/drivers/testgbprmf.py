"""GBPRMF driver (src/models/pl/testgbprmf.py:19-113): same globals and worker."""
import os

from ..gbprmf import GBPRMF
from ..sampler_gbpr import Sampler
from ._common import args, load_fold, run_folds

folds = 5
binarize_threshold = 3
gsize = 1
rho = .4
reg = .01
topN = 100
split_method = 'cv'
eval_metrics = ['pre', 'recall', 'map', 'mrr', 'ndcg']
n_factors = 100
batch_size = 100
negSample = 5


def worker(fold, n_users, n_items, dataset_dir):
    trasR, tstsR = load_fold(dataset_dir, fold, n_users, n_items, binarize_threshold)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1), trasR.shape, trasR.nnz,
          '%.2f' % (trasR.nnz / float(trasR.shape[0])))
    sampler = Sampler(trasR, gsize, negSample, batch_size)
    gbprmf = GBPRMF(n_users, n_items, topN, rho, gsize, split_method, eval_metrics, reg,
                    n_factors, batch_size, device=int(os.environ.get("CF_DEVICE", "0")))
    scores = gbprmf.train(fold + 1, trasR, tstsR, sampler)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1), 'gsize=', gsize, 'rho=', rho,
          'reg=', reg)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1),
          ','.join(['%s' % m for m in eval_metrics]) + '@%d=' % topN +
          ','.join(['%.6f' % s for s in scores]))
    gbprmf.close()
    sampler.close()
    return scores


if __name__ == '__main__':
    print('gsize=', gsize, 'rho=', rho, 'reg=', reg)
    dataset_dir, nfolds, parallel = args(5)
    run_folds(worker, 943, 1682, dataset_dir, nfolds, topN, eval_metrics, parallel)
