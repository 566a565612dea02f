"""CPLR driver (src/models/pl/testcplr_u.py): same globals and worker."""
import os

from ..cplr import CPLR
from ._common import args, load_fold, run_folds

folds = 5
binarize_threshold = 3
topK = 200
reg = .1
topN = 100
split_method = 'cv'
eval_metrics = ['pre', 'recall', 'map', 'mrr', 'ndcg']
alpha = 1.
beta = 1.
gamma = 1.
n_factors = 100
batch_size = 100
max_iter = 50


def worker(fold, n_users, n_items, dataset_dir):
    trasR, tstsR = load_fold(dataset_dir, fold, n_users, n_items, binarize_threshold)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1), trasR.shape, trasR.nnz,
          '%.2f' % (trasR.nnz / float(trasR.shape[0])))
    cplr = CPLR(n_users, n_items, topK, topN, split_method, eval_metrics, alpha, beta, gamma, reg,
                n_factors, batch_size, max_iter=max_iter,
                device=int(os.environ.get("CF_DEVICE", "0")))
    scores = cplr.train(fold + 1, trasR, tstsR)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1),
          ','.join(['%s' % m for m in eval_metrics]) + '@%d=' % topN +
          ','.join(['%.6f' % s for s in scores]))
    cplr.close()
    return scores


if __name__ == '__main__':
    print('topK=', topK, 'reg=', reg)
    dataset_dir, nfolds, parallel = args(1)
    run_folds(worker, 943, 1682, dataset_dir, nfolds, topN, eval_metrics, parallel)
