"""GPU parity of the recommend step (bprmf.py:77-103 and siblings): scores,
train-item exclusion and top-k order (descending, ties to the lower id, TF
TopKV2) against the oracle's literal restatement.  Every test runs on both
fused kernels (cf_set_option fused_variant: the sequential one and the
software-pipelined one and, round 5, the specialised-wave one and the
128-users-per-block one)."""
import numpy as np
import pytest

from oracle import cf_oracle as O

pytestmark = pytest.mark.gpu

_FV = [0]


@pytest.fixture(autouse=True, params=[0, 1, 2, 3], ids=["fused-seq", "fused-pipe", "fused-ws", "fused-u128"])
def fused_variant(request):
    _FV[0] = request.param
    yield request.param
    _FV[0] = 0


def setup(model, fold1, d, seed, bias=False, truncated=True):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    e = Engine(model, nu, ni, d, n_neg=1, gsize=1, seed=1)
    e.set_option("fused_variant", _FV[0])
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    rng = np.random.RandomState(seed)
    U = O.init_table(rng, (nu, d), truncated=truncated)
    V = O.init_table(rng, (ni, d), truncated=truncated)
    e.set_table("user", U)
    e.set_table("item", V)
    b = None
    if bias:
        b = O.init_table(rng, (ni,))
        e.set_table("bias", b)
    return e, U, V, b


def check_lists(gpu_idx, scores, oracle_lists, atol):
    """Exact order, except that adjacent near-ties (|ds| <= atol in the oracle's
    fp64 scores) may swap because fp32 summation order differs."""
    for r, (g, o) in enumerate(zip(gpu_idx, oracle_lists)):
        g = [int(x) for x in g if x >= 0]
        assert len(g) == len(o), r
        if g == o:
            continue
        s = scores[r]
        for a, b in zip(g, o):
            if a != b:
                assert abs(s[a] - s[b]) <= atol, (r, a, b, s[a], s[b])


@pytest.mark.parametrize("path", [0, 1])          # auto (fused MFMA for k <= 28), materialised
@pytest.mark.parametrize("model,d", [("bpr", 32), ("gbpr", 20), ("cml", 50), ("amf", 100),
                                     ("bpr", 128), ("cml", 7)])
def test_topk_matches_oracle(fold1, model, d, path):
    e, U, V, b = setup(model, fold1, d, 21, bias=(model == "gbpr"), truncated=(model != "cml"))
    e.set_option("topk_path", path)
    tst_ip = fold1["test_indptr"]
    users = np.nonzero(np.diff(tst_ip))[0].astype(np.int32)
    for k in (1, 10, 28, 32, 100):
        idx = e.score_topk(users, k, exclude_train=True)
        S = O.predict(model, U.astype(np.float64), V.astype(np.float64),
                      None if b is None else b.astype(np.float64), users)
        ref = O.recommend(S, fold1["train_indptr"], fold1["train_indices"], users, k)
        check_lists(idx, S, ref, atol=1e-5)
    e.close()


def test_recommend_equals_literal_overfetch(fold1):
    """Excluding train items before top-k == the reference's top_k over
    max|train|+topN followed by the python filter loop (bprmf.py:90-103)."""
    e, U, V, _ = setup("bpr", fold1, 16, 22)
    users = np.arange(0, 943, 7, dtype=np.int32)
    S = O.predict("bpr", U.astype(np.float64), V.astype(np.float64), None, users)
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    sets = [set(ix[ip[u]:ip[u + 1]].tolist()) for u in users]
    lit = O.recommend_literal(S, sets, 10)
    idx = e.score_topk(users, 10)
    check_lists(idx, S, lit, atol=1e-5)
    e.close()


@pytest.mark.parametrize("path", [1, 2])
def test_ties_go_to_lower_id(fold1, path):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    e = Engine("bpr", nu, ni, 4, seed=1)
    e.set_option("fused_variant", _FV[0])
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    U = np.ones((nu, 4), np.float32)
    V = np.zeros((ni, 4), np.float32)
    V[::3] = 1.0   # every third item ties at score 4, the rest tie at 0
    e.set_table("user", U)
    e.set_table("item", V)
    e.set_option("topk_path", path)
    idx, val = e.score_topk(np.array([5], np.int32), 28, exclude_train=False, return_values=True)
    assert list(idx[0]) == list(range(0, 84, 3))
    assert np.all(val[0] == 4.0)
    if path == 1:
        idx = e.score_topk(np.array([5], np.int32), 600, exclude_train=False)
        assert list(idx[0][:561]) == list(range(0, ni, 3))
        assert list(idx[0][561:600]) == [x for x in range(ni) if x % 3][:39]
    # many users at once (several fused blocks), all tied
    idx = e.score_topk(np.arange(0, 943, 3, dtype=np.int32), 20, exclude_train=False)
    assert all(list(r) == list(range(0, 60, 3)) for r in idx)
    e.close()


@pytest.mark.parametrize("path", [1, 2])
def test_exclusion_and_padding(fold1, path):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    # tiny graph: user 0 owns items 0..7 of 10 -> only 2 items remain
    ip = np.array([0, 8, 9], np.int64)
    ix = np.array(list(range(8)) + [3], np.int32)
    e = Engine("bpr", 2, 10, 4, seed=1)
    e.set_option("fused_variant", _FV[0])
    e.set_interactions(ip, ix)
    rng = np.random.RandomState(0)
    e.set_table("user", rng.randn(2, 4).astype(np.float32))
    e.set_table("item", rng.randn(10, 4).astype(np.float32))
    e.set_option("topk_path", path)
    idx = e.score_topk(np.array([0, 1], np.int32), 5)
    assert sorted(int(x) for x in idx[0][:2]) == [8, 9]
    assert list(idx[0][2:]) == [-1, -1, -1]
    assert 3 not in idx[1] and len(set(idx[1].tolist())) == 5
    e.close()


def _excl_csr(fold1, n_users, item_mask, with_train):
    """Per-user excluded items as a CSR (oracle.recommend's train argument):
    the flagged items, plus the user's train items when with_train."""
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    flagged = np.nonzero(item_mask)[0]
    rows = []
    for u in range(n_users):
        s = set(flagged.tolist())
        if with_train:
            s |= set(ix[ip[u]:ip[u + 1]].tolist())
        rows.append(np.array(sorted(s), np.int32))
    indptr = np.zeros(n_users + 1, np.int64)
    indptr[1:] = np.cumsum([len(r) for r in rows])
    return indptr, np.concatenate(rows)


@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("model,d", [("bpr", 32), ("gbpr", 64), ("cml", 50)])
def test_topk_item_mask_matches_oracle(fold1, model, d, path):
    """cf_score_topk's mask_or_NULL and cf_score_topk_ex's
    item mask: flagged items are dropped for every user -- on top of the
    train items (exclude_train) or alone (cf_score_topk with a mask) -- on the
    fused kernels (k <= 28 and the wide lists) and the materialised path."""
    e, U, V, b = setup(model, fold1, d, 23, bias=(model == "gbpr"), truncated=(model != "cml"))
    e.set_option("topk_path", path)
    rng = np.random.RandomState(5)
    mask = (rng.rand(int(fold1["n_items"])) < 0.2).astype(np.uint8)
    mask[:70] = 1                       # whole 64-item tiles flagged too
    users = np.arange(0, 943, 5, dtype=np.int32)
    S = O.predict(model, U.astype(np.float64), V.astype(np.float64),
                  None if b is None else b.astype(np.float64), users)
    both = _excl_csr(fold1, 943, mask, True)
    alone = _excl_csr(fold1, 943, mask, False)
    for k in (10, 100):
        idx = e.score_topk(users, k, exclude_train=True, item_mask=mask)
        check_lists(idx, S, O.recommend(S, both[0], both[1], users, k), atol=1e-5)
        idx = e.recommend(users, k, mask=mask)
        check_lists(idx, S, O.recommend(S, alone[0], alone[1], users, k), atol=1e-5)
        idx = e.recommend(users, k)     # NULL: the reference's train filter
        check_lists(idx, S, O.recommend(S, fold1["train_indptr"], fold1["train_indices"], users, k),
                    atol=1e-5)
    e.close()


def test_wide_k_takes_fused_path(fold1):
    """GBPR's topN = 100 (testgbprmf.py:23-32) streams through the fused
    kernel's wide lists (no score matrix written: no score launch)."""
    e, U, V, b = setup("gbpr", fold1, 64, 24, bias=True)
    users = np.arange(943, dtype=np.int32)
    e.profile_reset()
    e.profile(True)
    e.score_topk(users, 100)
    e.profile(False)
    assert e.profile_read("score")[1] == 0
    assert e.profile_read("topk")[1] == 1
    e.close()


@pytest.mark.parametrize("k", [100, 128])
def test_wide_k_gbpr_million_items(k):
    """k = 100 / 128 with GBPR's +b at d = 64 over 1M items (cfg4's item
    count, where the materialised path would write [chunk, 1M] score rows):
    128 users against the float64 oracle under the near-tie rule."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni, d = 512, 1_000_000, 64
    rng = np.random.RandomState(31)
    deg = rng.randint(1, 60, nu)
    ip = np.zeros(nu + 1, np.int64)
    ip[1:] = np.cumsum(deg)
    ix = np.concatenate([np.sort(rng.choice(ni, g, replace=False)) for g in deg]).astype(np.int32)
    e = Engine("gbpr", nu, ni, d, n_neg=1, gsize=1, seed=3)
    e.set_option("fused_variant", _FV[0])
    e.set_interactions(ip, ix)
    U = O.init_table(rng, (nu, d))
    V = O.init_table(rng, (ni, d))
    bb = O.init_table(rng, (ni,))
    e.set_table("user", U)
    e.set_table("item", V)
    e.set_table("bias", bb)
    users = np.arange(0, nu, 4, dtype=np.int32)
    e.profile_reset()
    e.profile(True)
    idx = e.score_topk(users, k)
    e.profile(False)
    assert e.profile_read("score")[1] == 0
    S = O.predict("gbpr", U.astype(np.float64), V.astype(np.float64), bb.astype(np.float64), users)
    check_lists(idx, S, O.recommend(S, ip, ix, users, k), atol=2e-5)
    e.close()
