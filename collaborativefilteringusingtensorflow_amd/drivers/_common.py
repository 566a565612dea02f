"""Fold loop shared by the drivers (testbprmf.py:55-125 and siblings).

The reference runs folds in a ``multiprocessing.Pool`` of forked processes.
A forked child must not inherit an initialised HIP runtime, so folds here run
either sequentially in this process or in *spawned* processes, fold k on HIP
device k % n_devices.
"""
import multiprocessing
import sys

import numpy as np


def run_folds(worker, n_users, n_items, dataset_dir, folds, topN, eval_metrics, parallel=False):
    if parallel:
        ctx = multiprocessing.get_context("spawn")
        with ctx.Pool(processes=folds) as pool:
            results = [pool.apply_async(worker, (f, n_users, n_items, dataset_dir))
                       for f in range(folds)]
            scores = np.array([r.get() for r in results])
    else:
        scores = np.array([worker(f, n_users, n_items, dataset_dir) for f in range(folds)])
    aves = scores.sum(0) / len(scores)
    stds = np.sqrt(np.power(scores - aves, 2).sum(0) / len(scores))
    print('ave@' + str(topN) + '=[' + ','.join(['%.4f' % a for a in aves]) + ']',
          'std@' + str(topN) + '=[' + ','.join(['%.4f' % s for s in stds]) + ']')
    sys.stdout.flush()
    return aves, stds


def args(default_folds):
    dataset_dir = sys.argv[1] if len(sys.argv) > 1 else "data/movielens/ml-100k/"
    if not dataset_dir.endswith("/"):
        dataset_dir += "/"
    folds = int(sys.argv[2]) if len(sys.argv) > 2 else default_folds
    parallel = "--parallel" in sys.argv
    return dataset_dir, folds, parallel


def load_fold(dataset_dir, fold, n_users, n_items, binarize_threshold):
    from scipy.sparse import lil_matrix
    from ..io_util import loadSparseR, matBinarize
    tra = lil_matrix(matBinarize(loadSparseR(n_users, n_items, dataset_dir + 'ratings__' +
                                             str(fold + 1) + '_tra.txt'), binarize_threshold))
    tst = lil_matrix(matBinarize(loadSparseR(n_users, n_items, dataset_dir + 'ratings__' +
                                             str(fold + 1) + '_tst.txt'), binarize_threshold))
    return tra, tst
