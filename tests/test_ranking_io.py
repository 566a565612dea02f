"""Metrics and ingest pinned to outputs of the reference's own code
(tests/golden/ranking_cases.json, ioutil_cases.json, ml100k_fold1.npz --
all produced by tests/golden/make_golden.py importing the reference)."""
import json
import os

import numpy as np
import pytest

from collaborativefilteringusingtensorflow_amd import ranking as R
from collaborativefilteringusingtensorflow_amd import io_util as IO

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("case", load("ranking_cases.json"), ids=lambda c: c["tag"])
def test_metrics_match_reference(case):
    if case["kind"] == "cv":
        yt = [set(t) for t in case["yss_true"]]
        got = R.evaluateCV(yt, case["yss_pred"], case["metrics"], case["k"])
    else:
        got = R.evaluateLOOV(case["ys_true"], case["yss_pred"], case["metrics"], case["k"])
    np.testing.assert_allclose(got, case["expected"], rtol=1e-12, atol=1e-15)


def test_nonstandard_ndcg_known_answer():
    # ranking.py:125: standard NDCG@3 would give 0.4732 here
    yt = [set([4, 2]), set([3, 1]), set([1])]
    yp = [[3, 1, 2], [1, 2], [2, 3, 1]]
    assert abs(R.ndcg_k_score(yt, yp, 3) - 2.0 / 3.0) < 1e-12


def test_metric_errors_like_reference():
    with pytest.raises(ValueError):
        R.precision_k_score([], [], 5)
    with pytest.raises(ValueError):
        R.ndcg_k_score([set([1])], [[1]], 0)
    with pytest.raises(ValueError):
        R.hr_k_score([1, 2], [[1]], 5)
    assert R.evaluateCV([set([1])], [[1]], ["pre", "bogus"], 1) == [1.0, None]


@pytest.mark.parametrize("case", load("ioutil_cases.json"), ids=lambda c: c["tag"])
def test_loader_matches_reference(case, tmp_path):
    p = tmp_path / "r.txt"
    p.write_text(case["text"])
    Rm = IO.loadSparseR(case["n_users"], case["n_items"], str(p))
    np.testing.assert_array_equal(Rm.toarray(), np.asarray(case["ratings"]))
    Bm = IO.matBinarize(Rm, case["threshold"])
    np.testing.assert_array_equal(Bm.toarray(), np.asarray(case["binary"]))
    assert IO.split_row(" a,b ;c\n") == ["a", "b ;c"]


def test_fold_fixture_roundtrip(fold1):
    import scipy.sparse as sp
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    M = sp.lil_matrix(sp.csr_matrix((np.ones(len(ix), np.float32), ix, ip), shape=(943, 1682)))
    ip2, ix2, shape = IO.to_csr(M)
    assert shape == (943, 1682)
    assert np.array_equal(ip2, ip) and np.array_equal(ix2, ix)
    assert len(ix) == 44243                        # nnz after > 3 binarisation
    assert len(np.nonzero(np.diff(fold1["test_indptr"]))[0]) == 919


def _reference_restatement(text, n_users, n_items):
    """Pure-Python restatement of IOUtil.loadSparseR (IOUtil.py:8-16) on
    Util.split_row (Util.py:5-11): dict of the last write per entry, zeros
    dropped, Python index wrap -- the checker for the native parser."""
    out = {}
    for line in text.splitlines(True):
        phs = IO.split_row(line)
        if len(phs) == 2:
            key, v = (int(phs[0]), int(phs[1])), 1.0
        elif len(phs) == 3:
            key, v = (int(phs[0]), int(phs[1])), float(phs[2])
        else:
            continue
        u, i = key
        u, i = (u + n_users if u < 0 else u), (i + n_items if i < 0 else i)
        assert 0 <= u < n_users and 0 <= i < n_items
        out[(u, i)] = v
    M = np.zeros((n_users, n_items))
    for (u, i), v in out.items():
        M[u, i] = v
    return M


@pytest.mark.parametrize("text", [
    "0 1 5\n0 1 0\n1 1 2\n",              # a later 0 removes the entry
    "-1 -2 4\n0 0 1\n",                    # Python negative-index wrap
    "\n\n  0\t2\t3.5 \r\n\n1 0\n",        # blank lines, CRLF, 2-field line = 1
    " 0 , 1 , 4.5 \n1;2;3\n",              # ',' fields keep blanks; ';' separator
    "0 1 4 5 6\n1\n0 0 nan\n1 1 inf\n",   # ignored field counts, nan / inf ratings
])
def test_native_loader_edge_cases(text, tmp_path):
    p = tmp_path / "r.txt"
    p.write_text(text)
    ref = _reference_restatement(text, 2, 3)
    got = IO.loadSparseR(2, 3, str(p)).toarray()
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_array_equal(np.nan_to_num(got), np.nan_to_num(ref))


@pytest.mark.parametrize("text", ["0 x 3\n", "5 0 1\n", "0 1 abc\n", "0,,1\n"])
def test_native_loader_rejects_like_reference(text, tmp_path):
    from collaborativefilteringusingtensorflow_amd._native import NativeError
    p = tmp_path / "r.txt"
    p.write_text(text)
    with pytest.raises(NativeError):
        IO.loadSparseR(3, 3, str(p))


def test_native_loader_multithreaded_last_write_wins(tmp_path):
    # ~3 MB: several parser threads; duplicates spread over the whole file
    rng = np.random.RandomState(0)
    n_users, n_items, n = 300, 200, 250000
    u = rng.randint(0, n_users, n)
    i = rng.randint(0, n_items, n)
    r = rng.randint(0, 6, n).astype(float) / 2
    seps = ["\t", " ", ","]
    lines = ["%d%s%d%s%g\n" % (a, seps[k % 3], b, seps[k % 3], c)
             for k, (a, b, c) in enumerate(zip(u, i, r))]
    text = "".join(lines)
    p = tmp_path / "big.txt"
    p.write_text(text)
    ref = _reference_restatement(text, n_users, n_items)
    got = IO.loadSparseR(n_users, n_items, str(p)).toarray()
    np.testing.assert_array_equal(got, ref)
    ip, ix = IO.load_csr(str(p), n_users, n_items, threshold=1.5)
    B = np.zeros_like(ref)
    for row in range(n_users):
        B[row, ix[ip[row]:ip[row + 1]]] = 1.0
    np.testing.assert_array_equal(B, (ref > 1.5).astype(float))
    assert all(np.all(np.diff(ix[ip[k]:ip[k + 1]]) > 0) for k in range(n_users))


def test_native_loader_fold_roundtrip(fold1, tmp_path):
    # the fold fixture written back as a rating file (train entries rated 4,
    # plus entries rated <= 3 that binarisation must drop) reloads exactly
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    rows = np.repeat(np.arange(943), np.diff(ip))
    rng = np.random.RandomState(1)
    extra = [(rng.randint(943), rng.randint(1682)) for _ in range(3000)]
    extra = [(a, b) for a, b in extra if b not in set(ix[ip[a]:ip[a + 1]].tolist())]
    lines = ["%d\t%d\t4\n" % (a, b) for a, b in zip(rows, ix)] + \
            ["%d\t%d\t%d\n" % (a, b, 1 + (a + b) % 3) for a, b in extra]
    order = rng.permutation(len(lines))
    p = tmp_path / "fold.txt"
    p.write_text("".join(lines[k] for k in order))
    ip2, ix2 = IO.load_csr(str(p), 943, 1682, threshold=3)
    assert np.array_equal(ip2, ip) and np.array_equal(ix2, ix)


def test_native_item_user_transpose_matches_numpy():
    """cf_synth_item_users (the sharded GBPR group source) equals the
    transpose of the synthetic user -> item CSR (distributed.item_users)."""
    from collaborativefilteringusingtensorflow_amd.engine import synth_graph, synth_item_users
    from collaborativefilteringusingtensorflow_amd.distributed import item_users
    nu, ni = 3000, 700
    ip, ix = synth_graph(nu, ni, 12.0, 0.8, 99, n_threads=3)
    tp, tu = item_users(ip, ix, ni)
    for nt in (1, 4):
        tp2, tu2 = synth_item_users(nu, ni, 12.0, 0.8, 99, n_threads=nt)
        np.testing.assert_array_equal(tp2, tp)
        np.testing.assert_array_equal(tu2, tu)
