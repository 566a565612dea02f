"""Ensemble driver, ensemble_ (W negatives) variant (src/models/pl/testensemble_.py):
same globals and worker, fed by the sampler_ranking drop-in."""
import os

from ..ensemble_ import Ensemble
from ..sampler_ranking import Sampler
from ._common import args, load_fold, run_folds

folds = 5
binarize_threshold = 3
reg = .1
kensemble = 5
topN = 10
split_method = 'cv'
eval_metrics = ['pre', 'recall', 'map', 'mrr', 'ndcg']
n_factors = 100
batch_size = 100
negSample = 5


def worker(fold, n_users, n_items, dataset_dir):
    trasR, tstsR = load_fold(dataset_dir, fold, n_users, n_items, binarize_threshold)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1), trasR.shape, trasR.nnz,
          '%.2f' % (trasR.nnz / float(trasR.shape[0])))
    device = int(os.environ.get("CF_DEVICE", "0"))
    sampler = Sampler(trasR=trasR, n_neg=negSample, batch_size=batch_size, device=device)
    en = Ensemble(n_users, n_items, kensemble, topN, split_method, eval_metrics, reg, n_factors,
                  batch_size, device=device)
    scores = en.train(fold + 1, trasR, tstsR, sampler)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1),
          ','.join(['%s' % m for m in eval_metrics]) + '@%d=' % topN +
          ','.join(['%.6f' % s for s in scores]))
    en.close()
    sampler.close()
    return scores


if __name__ == '__main__':
    print('reg=', reg, 'kensemble=', kensemble)
    dataset_dir, nfolds, parallel = args(1)
    run_folds(worker, 943, 1682, dataset_dir, nfolds, topN, eval_metrics, parallel)
