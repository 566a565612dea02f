"""Bit-exact host sampler mode (csrc/cf_mt_sampler.cpp).

Pinned two ways:
* against the reference's OWN batch streams (tests/golden/sampler_streams.npz,
  captured by tests/golden/make_golden.py from src/samplers/*.py after
  ``np.random.seed(s)``): the first 40 batches must be identical;
* against a numpy-literal restatement of the reference producer loop (the
  same RandomState calls in the same order) across several epochs, which
  exercises the in-place re-shuffle of every epoch.
Host-only: needs the built library, no GPU.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from collaborativefilteringusingtensorflow_amd import sampler_gbpr, sampler_ranking, sampler_uij_ranking

SEEDS = {"rank_b100_w1": 11, "rank_b100_w5": 12, "rank_b50_w5": 13, "uij_b100": 14,
         "gbpr_b100_g1_w5": 15, "gbpr_b100_g3_w2": 16}


def _tra(fold1):
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    return sp.lil_matrix(sp.csr_matrix((np.ones(len(ix), np.float32), ix, ip), shape=(943, 1682)))


@pytest.mark.parametrize("name", sorted(SEEDS))
def test_exact_sampler_reproduces_reference_stream(fold1, streams, name):
    tra = _tra(fold1)
    P = streams[name + "/pairs"]
    Ng = streams[name + "/negs"]
    B, W = P.shape[1], Ng.shape[2]
    if name.startswith("rank"):
        s = sampler_ranking.ExactSampler(tra, n_neg=W, batch_size=B, seed=SEEDS[name])
    elif name.startswith("uij"):
        s = sampler_uij_ranking.ExactSampler(tra, batch_size=B, seed=SEEDS[name])
    else:
        G = streams[name + "/groups"].shape[2]
        s = sampler_gbpr.ExactSampler(tra, gsize=G, n_neg=W, batch_size=B, seed=SEEDS[name])
    for b in range(P.shape[0]):
        out = s.next_batch()
        if name.startswith("uij"):
            assert out.dtype == np.int64 and out.shape == (B, 3)
            np.testing.assert_array_equal(out[:, :2], P[b])
            np.testing.assert_array_equal(out[:, 2:], Ng[b])
            continue
        np.testing.assert_array_equal(out[0], P[b])
        np.testing.assert_array_equal(out[1], Ng[b])
        if name.startswith("gbpr"):
            np.testing.assert_array_equal(out[2], streams[name + "/groups"][b])
    s.close()


def _numpy_producer(tra, B, W, G, seed, n_batches):
    """The reference producer loop (sampler_ranking.py:22-37 /
    sampler_gbpr.py:23-43) on numpy's legacy global RandomState."""
    np.random.seed(seed)
    pairs = np.array(tra.nonzero()).T
    pos = {u: set(r) for u, r in enumerate(tra.rows)}
    cols = {i: list(c) for i, c in enumerate(tra.transpose().rows)}
    n_users, n_items = tra.shape
    out = []
    while len(out) < n_batches:
        np.random.shuffle(pairs)
        for i in range(int(len(pairs) / B)):
            pb = pairs[i * B:(i + 1) * B, :].copy()
            nb = np.random.randint(0, n_items, size=(len(pb), W))
            gb = np.random.randint(0, n_users, size=(len(pb), G)) if G else None
            for k, (u, it) in enumerate(pb):
                for j in range(W):
                    while nb[k, j] in pos[u]:
                        nb[k, j] = np.random.randint(0, n_items)
                if G:
                    gb[k] = np.random.choice(cols[it], G)
            out.append((pb, nb, gb))
            if len(out) == n_batches:
                break
    return out


@pytest.mark.parametrize("G", [0, 2])
def test_exact_sampler_matches_numpy_across_epochs(G):
    rng = np.random.RandomState(3)
    n_users, n_items = 40, 300
    M = sp.lil_matrix((n_users, n_items), dtype=np.float32)
    for u in range(n_users):
        for it in rng.choice(n_items, rng.randint(1, 25), replace=False):
            M[u, it] = 1.0
    B, W, seed = 37, 3, 2026
    nnz = M.nnz
    n_batches = 3 * (nnz // B) + 2                 # three re-shuffles
    ref = _numpy_producer(M, B, W, G, seed, n_batches)
    if G:
        s = sampler_gbpr.ExactSampler(M, gsize=G, n_neg=W, batch_size=B, seed=seed)
    else:
        s = sampler_ranking.ExactSampler(M, n_neg=W, batch_size=B, seed=seed)
    for pb, nb, gb in ref:
        out = s.next_batch()
        np.testing.assert_array_equal(out[0], pb)
        np.testing.assert_array_equal(out[1], nb)
        if G:
            np.testing.assert_array_equal(out[2], gb)
    assert s.state() == (3, 2)
    s.close()


def test_exact_sampler_rejects_like_numpy():
    M = sp.lil_matrix((3, 5), dtype=np.float32)
    M[0, 1] = 1.0
    with pytest.raises(ValueError):
        sampler_ranking.ExactSampler(M, seed=2 ** 32)
