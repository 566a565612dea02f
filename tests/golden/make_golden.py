"""Generate the committed golden fixtures from the *reference itself*.

Test infrastructure only.  Runs in the build container, where the read-only
reference checkout lives at /root/reference; the GPU box never runs this
script (it only reads the .npz/.json files it wrote).

What is captured, and from which reference code:

* ``ml100k_fold1.npz`` -- fold-1 train/test matrices of ml-100k, loaded with
  ``src/utils/IOUtil.py:loadSparseR`` (IOUtil.py:23-32) and binarised with
  ``src/utils/Util.py:matBinarize`` (Util.py:15-16) at threshold 3, exactly as
  ``src/models/pl/testbprmf.py:33-40`` does.  Stored as CSR (indptr/indices).
* ``sampler_streams.npz`` -- the first batches of the three hot-path samplers
  (``sampler_ranking.py:22-37``, ``sampler_uij_ranking.py:22-38``,
  ``sampler_gbpr.py:23-43``), seeded with ``np.random.seed`` immediately
  before construction and captured on the CONSUMER side of ``next_batch()``
  (stay inside the first epoch, so the last-batch race never
  appears in a fixture).
* ``ranking_cases.json`` -- known answers of ``src/metrics/ranking.py``
  (the __main__ demo cases at :124-131, the LOOV case, and seeded random
  cases), computed by calling the reference functions.
* ``ioutil_cases.json`` -- small text inputs run through ``loadSparseR`` /
  ``matBinarize`` to pin the separator / field-count / threshold rules.

Each sampler capture runs in a child process because the reference samplers
start non-daemon ``while True`` threads; the child ends with ``os._exit``.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
DATA = REF + "/data/movielens/ml-100k/"


def _ref_paths():
    for sub in ("src/utils", "src/samplers", "src/metrics"):
        p = os.path.join(REF, sub)
        if p not in sys.path:
            sys.path.insert(0, p)


def load_fold(fold=1):
    _ref_paths()
    from IOUtil import loadSparseR
    from Util import matBinarize
    from scipy.sparse import lil_matrix
    tra = lil_matrix(matBinarize(loadSparseR(943, 1682, DATA + "ratings__%d_tra.txt" % fold), 3))
    tst = lil_matrix(matBinarize(loadSparseR(943, 1682, DATA + "ratings__%d_tst.txt" % fold), 3))
    return tra, tst


# (name, sampler module, seed, kwargs, n_batches)
STREAMS = [
    ("rank_b100_w1", "sampler_ranking", 11, dict(n_neg=1, batch_size=100), 40),
    ("rank_b100_w5", "sampler_ranking", 12, dict(n_neg=5, batch_size=100), 40),
    ("rank_b50_w5", "sampler_ranking", 13, dict(n_neg=5, batch_size=50), 40),
    ("uij_b100", "sampler_uij_ranking", 14, dict(batch_size=100), 40),
    ("gbpr_b100_g1_w5", "sampler_gbpr", 15, dict(gsize=1, n_neg=5, batch_size=100), 40),
    ("gbpr_b100_g3_w2", "sampler_gbpr", 16, dict(gsize=3, n_neg=2, batch_size=100), 40),
]


def capture_child(name, out_path):
    """Child process: seed, build the reference sampler, pull batches."""
    spec = {s[0]: s for s in STREAMS}[name]
    _, mod, seed, kwargs, nb = spec
    tra, _ = load_fold(1)
    np.random.seed(seed)
    sampler = __import__(mod).Sampler(tra, **kwargs)
    batches = [sampler.next_batch() for _ in range(nb)]
    if mod == "sampler_uij_ranking":
        arr = np.stack([np.asarray(b) for b in batches])          # [N,B,3] int64
        np.savez(out_path, pairs=arr[:, :, :2].astype(np.int32),
                 negs=arr[:, :, 2:].astype(np.int32), uij=arr)
    elif mod == "sampler_gbpr":
        np.savez(out_path,
                 pairs=np.stack([b[0] for b in batches]).astype(np.int32),
                 negs=np.stack([b[1] for b in batches]).astype(np.int32),
                 groups=np.stack([b[2] for b in batches]).astype(np.int32))
    else:
        np.savez(out_path,
                 pairs=np.stack([b[0] for b in batches]).astype(np.int32),
                 negs=np.stack([b[1] for b in batches]).astype(np.int32))
    sys.stdout.flush()
    os._exit(0)


def make_fold_fixture():
    tra, tst = load_fold(1)
    out = {}
    for tag, m in (("train", tra), ("test", tst)):
        csr = m.tocsr()
        csr.sort_indices()
        out[tag + "_indptr"] = csr.indptr.astype(np.int64)
        out[tag + "_indices"] = csr.indices.astype(np.int32)
    out["n_users"] = np.int64(943)
    out["n_items"] = np.int64(1682)
    # the exact pair order of trasR.nonzero() (sampler_ranking.py:13)
    nz = np.array(tra.nonzero()).T
    assert np.array_equal(nz[:, 0], np.repeat(np.arange(943), np.diff(out["train_indptr"])))
    assert np.array_equal(nz[:, 1], out["train_indices"])
    np.savez_compressed(os.path.join(HERE, "ml100k_fold1.npz"), **out)
    return tra


def make_streams():
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for spec in STREAMS:
            name = spec[0]
            path = os.path.join(td, name + ".npz")
            subprocess.check_call([sys.executable, __file__, "--capture", name, path], timeout=300)
            with np.load(path) as z:
                for k in z.files:
                    if k == "uij":
                        continue
                    res[name + "/" + k] = z[k]
    np.savez_compressed(os.path.join(HERE, "sampler_streams.npz"), **res)


def make_ranking_cases():
    _ref_paths()
    import ranking as R
    cases = []

    def cv_case(tag, yt, yp, k):
        metrics = ["pre", "recall", "map", "mrr", "ndcg"]
        cases.append(dict(tag=tag, kind="cv", k=k,
                          yss_true=[sorted(int(x) for x in s) for s in yt],
                          yss_pred=[[int(x) for x in p] for p in yp],
                          metrics=metrics,
                          expected=[float(v) for v in R.evaluateCV(yt, yp, metrics, k)]))

    # ranking.py:125-128
    cv_case("KA1", [set([4, 2]), set([3, 1]), set([1])], [[3, 1, 2], [1, 2], [2, 3, 1]], 3)
    # ranking.py:130-131 (assigned there but never printed)
    for k in (5, 10, 20):
        cv_case("KA2_k%d" % k, [set([0, 1, 3, 4, 5, 8, 10, 12, 16, 18])], [list(range(20))], k)
    # LOOV (hr/arhr return sums)
    cases.append(dict(tag="LOOV", kind="loov", k=2, ys_true=[2, 5, 7],
                      yss_pred=[[1, 2, 3], [5, 4], [0, 1]], metrics=["hr", "arhr"],
                      expected=[float(v) for v in R.evaluateLOOV([2, 5, 7], [[1, 2, 3], [5, 4], [0, 1]],
                                                               ["hr", "arhr"], 2)]))
    rng = np.random.RandomState(2024)
    for c in range(24):
        n_users = int(rng.randint(1, 30))
        n_items = int(rng.randint(5, 60))
        k = int(rng.choice([1, 3, 5, 10, 20]))
        yt, yp = [], []
        for _ in range(n_users):
            nt = int(rng.randint(1, 12))
            yt.append(set(int(x) for x in rng.choice(n_items, size=min(nt, n_items), replace=False)))
            npred = int(rng.randint(0, k + 5))
            yp.append([int(x) for x in rng.choice(n_items, size=min(npred, n_items), replace=False)])
        cv_case("rand%02d" % c, yt, yp, k)
        ys = [int(rng.randint(0, n_items)) for _ in range(n_users)]
        cases.append(dict(tag="loov_rand%02d" % c, kind="loov", k=k, ys_true=ys,
                          yss_pred=yp, metrics=["hr", "arhr"],
                          expected=[float(v) for v in R.evaluateLOOV(ys, yp, ["hr", "arhr"], k)]))
    with open(os.path.join(HERE, "ranking_cases.json"), "w") as f:
        json.dump(cases, f, indent=0)


IO_TEXTS = [
    ("tabs_3field", "0\t1\t4.0\n2\t3\t2.5\n1\t0\t3.0\n", 3, 4, 3),
    ("comma", "0,1,5\n1,2,1\n2,0,4\n", 3, 3, 3),
    ("semicolon", "0;0;4\n1;1;3.5\n", 2, 2, 3),
    ("two_field", "0 1\n1 2\n2 0\n", 3, 3, 0),
    ("mixed_ignored_4field", "0 1 4 881250949\n1 1 5\n2 2\n", 3, 3, 3),
    ("dup_last_wins", "0 1 2\n0 1 5\n1 0 4\n", 2, 2, 3),
]


def make_io_cases():
    _ref_paths()
    from IOUtil import loadSparseR
    from Util import matBinarize
    cases = []
    with tempfile.TemporaryDirectory() as td:
        for tag, text, nu, ni, thr in IO_TEXTS:
            p = os.path.join(td, tag + ".txt")
            with open(p, "w") as f:
                f.write(text)
            R = loadSparseR(nu, ni, p)
            B = matBinarize(R, thr)
            cases.append(dict(tag=tag, text=text, n_users=nu, n_items=ni, threshold=thr,
                              ratings=R.toarray().tolist(),
                              binary=B.toarray().tolist()))
    with open(os.path.join(HERE, "ioutil_cases.json"), "w") as f:
        json.dump(cases, f, indent=0)


if __name__ == "__main__":
    if len(sys.argv) == 4 and sys.argv[1] == "--capture":
        capture_child(sys.argv[2], sys.argv[3])
    make_fold_fixture()
    make_streams()
    make_ranking_cases()
    make_io_cases()
    print("golden fixtures written to", HERE)
