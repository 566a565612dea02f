"""AMF driver (src/models/others/testamf.py:19-130): same globals and worker."""
import os

from ..amf import AMF
from ..sampler_ranking import Sampler
from ._common import args, load_fold, run_folds

folds = 5
binarize_threshold = 3
epsilon = 1.
reg_adv = 1.
adv_method = "grad"
reg = .05
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
    sampler = Sampler(trasR=trasR, n_neg=negSample, batch_size=batch_size)
    amf = AMF(n_users, n_items, topN, split_method, eval_metrics, epsilon, reg_adv, adv_method,
              reg, n_factors, batch_size, device=int(os.environ.get("CF_DEVICE", "0")))
    scores = amf.train(fold + 1, trasR, tstsR, sampler)
    print(dataset_dir.split('/')[-2] + '@%d:' % (fold + 1),
          ','.join(['%s' % m for m in eval_metrics]) + '@%d=' % topN +
          ','.join(['%.6f' % s for s in scores]))
    amf.close()
    sampler.close()
    return scores


if __name__ == '__main__':
    print('epsilon=', epsilon, 'reg_adv=', reg_adv, 'adv_method=', adv_method, 'reg=', reg)
    dataset_dir, nfolds, parallel = args(1)
    run_folds(worker, 943, 1682, dataset_dir, nfolds, topN, eval_metrics, parallel)
