"""Fold loop shared by the drivers (testbprmf.py:55-125 and siblings).

The reference runs folds in a ``multiprocessing.Pool`` of forked processes
(testbprmf.py:113-125).  Here the folds are independent GPU replicas (SURVEY
8(f) row 2): with ``parallel`` each fold runs in its own *spawned* process
(a forked child must not inherit an initialised HIP runtime) pinned to HIP
device fold % n_devices through CF_DEVICE, so 5 folds train concurrently on a
node's GPUs; otherwise they run one after another in this process.  The
report is the reference's ave@N / std@N line.
"""
import multiprocessing
import os
import sys

import numpy as np


def _fold_entry(worker, fold, device, n_users, n_items, dataset_dir, q):
    os.environ["CF_DEVICE"] = str(device)
    try:
        q.put((fold, list(worker(fold, n_users, n_items, dataset_dir)), None))
    except BaseException as ex:  # reported to the parent, which raises
        q.put((fold, None, "%s: %s" % (type(ex).__name__, ex)))


def run_folds(worker, n_users, n_items, dataset_dir, folds, topN, eval_metrics, parallel=False,
              n_devices=None):
    if parallel:
        if n_devices is None:
            from .. import _native as N
            n_devices = max(1, N.device_count())
        ctx = multiprocessing.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_fold_entry,
                             args=(worker, f, f % n_devices, n_users, n_items, dataset_dir, q))
                 for f in range(folds)]
        for p in procs:
            p.start()
        got = {}
        for _ in range(folds):
            f, sc, err = q.get()
            if err is not None:
                for p in procs:
                    p.join()
                raise RuntimeError("fold %d failed: %s" % (f + 1, err))
            got[f] = sc
        for p in procs:
            p.join()
        scores = np.array([got[f] for f in range(folds)])
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
