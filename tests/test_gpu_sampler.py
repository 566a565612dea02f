"""Statistical / structural parity of the on-device sampler with the
reference samplers (sampler_ranking.py:22-37, sampler_uij_ranking.py:22-38,
sampler_gbpr.py:23-43).  The reference stream is unseeded numpy MT19937, so
parity is on the facts every reference batch satisfies:

* every negative j is NOT a positive of u (also checked on the captured
  reference batches: tests/test_golden_fixtures.py);
* each epoch draws floor(nnz/B) batches of distinct train pairs;
* negatives are uniform over the complement of Pos(u) (chi-square);
* group users are positives of the item (g in Pos^-1(i));
* same seed => same stream.
"""
import numpy as np
import pytest
from scipy import stats

pytestmark = pytest.mark.gpu


def csr_sets(indptr, indices):
    return [set(indices[indptr[u]:indptr[u + 1]].tolist()) for u in range(len(indptr) - 1)]


def make_csr_matrix(fold1):
    import scipy.sparse as sp
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    return sp.csr_matrix((np.ones(len(ix), np.float32), ix, ip), shape=(nu, ni))


def test_sampler_ranking_protocol_and_validity(fold1):
    from collaborativefilteringusingtensorflow_amd.sampler_ranking import Sampler
    R = make_csr_matrix(fold1)
    s = Sampler(R, n_neg=5, batch_size=100, seed=3)
    pos = csr_sets(fold1["train_indptr"], fold1["train_indices"])
    for _ in range(50):
        pairs, negs = s.next_batch()
        assert pairs.dtype == np.int32 and negs.dtype == np.int64
        assert pairs.shape == (100, 2) and negs.shape == (100, 5)
        for (u, i), js in zip(pairs, negs):
            assert i in pos[u]
            assert not any(int(j) in pos[u] for j in js)
    s.close()


def test_uij_protocol(fold1):
    from collaborativefilteringusingtensorflow_amd.sampler_uij_ranking import Sampler
    s = Sampler(make_csr_matrix(fold1), batch_size=64, seed=4)
    x = s.next_batch()
    assert x.shape == (64, 3) and x.dtype == np.int64
    s.close()


def test_epoch_is_a_permutation(fold1):
    from collaborativefilteringusingtensorflow_amd.sampler_ranking import Sampler
    B = 100
    nnz = len(fold1["train_indices"])
    per_epoch = nnz // B
    s = Sampler(make_csr_matrix(fold1), n_neg=1, batch_size=B, seed=5)
    for epoch in range(2):
        seen = []
        for _ in range(per_epoch):
            pairs, _ = s.next_batch()
            seen.append(pairs)
        seen = np.concatenate(seen)
        keys = seen[:, 0].astype(np.int64) * 1682 + seen[:, 1]
        assert len(np.unique(keys)) == per_epoch * B, epoch
        assert s.state() == (epoch, per_epoch)
    s.close()


@pytest.mark.parametrize("B", [100, 997, 4096])
def test_sorted_batches_same_sets_in_csr_order(fold1, B):
    """Sorted batches (cf_set_option "sorted_batches", the default since
    round 5): batch b of an epoch is the SAME set of pairs as the epoch
    bijection's slots [bB, bB + B) -- the draw only reads them in pair (CSR)
    order, i.e. ascending (u, i) -- over two epochs, with the order of the
    next epoch computed ahead on the engine's low-priority stream."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    per_epoch = len(ix) // B
    out = []
    for sb in (0, 1):
        e = Engine("bpr", nu, ni, 8, n_neg=1, seed=33)
        e.set_option("sorted_batches", sb)
        e.set_interactions(ip, ix)
        out.append([e.sample(B)[0] for _ in range(2 * per_epoch)])
        e.close()
    for b, (plain, srt) in enumerate(zip(*out)):
        kp = np.sort(plain[:, 0].astype(np.int64) * ni + plain[:, 1])
        ks = srt[:, 0].astype(np.int64) * ni + srt[:, 1]
        assert np.array_equal(np.sort(ks), kp), b          # the same batch set
        assert (np.diff(ks) > 0).all(), b                   # in CSR order
        ok = [(ix[ip[u]:ip[u + 1]] == i).any() for u, i in srt[:: max(1, B // 50)]]
        assert all(ok), b


@pytest.mark.parametrize("B", [100, 997])
def test_sorted_batches_with_records_equal_order_only(fold1, B):
    """sorted_batches 3 gathers each epoch's records in that order once, so
    the draw reads them coalesced: the same batches (pairs AND negatives,
    whose draws are keyed by slot) as sorted_batches 1, over two epochs."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    per_epoch = len(ix) // B
    out = []
    for sb in (1, 3):
        e = Engine("bpr", nu, ni, 8, n_neg=3, seed=34)
        e.set_option("sorted_batches", sb)
        e.set_interactions(ip, ix)
        out.append([e.sample(B)[:2] for _ in range(2 * per_epoch + 3)])
        e.close()
    for b, ((p1, n1), (p3, n3)) in enumerate(zip(*out)):
        assert np.array_equal(p1, p3) and np.array_equal(n1, n3), b


@pytest.mark.parametrize("sb", [1, 3], ids=["records", "index"])
@pytest.mark.parametrize("B", [20, 100, 997, 4096])
def test_epoch_counting_scatter_equals_radix_sort(fold1, sb, B):
    """The hand-written counting scatter that forms each epoch's order
    (cf_epoch.hip, cf_set_option("epoch_sort", 0), the default) gives the same
    batches as the stable radix sort it replaced (epoch_sort 1): bitwise the
    same pairs and negatives over two epochs, in both the records and the
    index form.  B = 20 has 2,213 batches per epoch, past kEpochMaxBins
    (1,024): both settings take the radix sort there."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    per_epoch = len(ix) // B
    n = 2 * per_epoch + 3 if B >= 100 else 40
    out = []
    for es in (0, 1):
        e = Engine("bpr", nu, ni, 8, n_neg=2, seed=36)
        e.set_option("sorted_batches", sb)
        e.set_option("epoch_sort", es)
        e.set_interactions(ip, ix)
        got = [e.sample(B)[:2] for _ in range(n)]
        if B < 100:   # the end of the epoch and the next one's start
            e.set_sampler_state(0, per_epoch - 3)
            got += [e.sample(B)[:2] for _ in range(6)]
        out.append(got)
        e.close()
    for b, ((p0, n0), (p1, n1)) in enumerate(zip(*out)):
        assert np.array_equal(p0, p1) and np.array_equal(n0, n1), b


@pytest.mark.parametrize("B", [1 << 16, 1 << 19, 3000])
def test_epoch_counting_scatter_large(B):
    """The same equality on a 2M-pair Zipf graph (the bijection's domain not a
    power of two, cycle walking on; 30 / 3 / 666 batches per epoch): the first
    batches, the last whole batch of the epoch and the first of the next."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine, synth_graph
    nu, ni = 70_000, 9_000
    ip, ix = synth_graph(nu, ni, 30.0, 0.8, 11, n_threads=8)
    per_epoch = len(ix) // B
    out = []
    for es in (0, 1):
        e = Engine("bpr", nu, ni, 8, n_neg=1, seed=37)
        e.set_option("sorted_batches", 1)
        e.set_option("epoch_sort", es)
        e.set_interactions(ip, ix)
        got = [e.sample(B)[0] for _ in range(2)]
        e.set_sampler_state(0, per_epoch - 1)
        got += [e.sample(B)[0] for _ in range(2)]
        out.append(got)
        e.close()
    for b, (p0, p1) in enumerate(zip(*out)):
        assert np.array_equal(p0, p1), b
        k = p0[:, 0].astype(np.int64) * ni + p0[:, 1]
        assert (np.diff(k) > 0).all(), b                     # CSR order inside the batch


@pytest.mark.parametrize("jump", [False, True], ids=["fresh", "state-jump"])
def test_side_stream_draw_waits_for_epoch_order(fold1, jump):
    """prep_stream 1 draws on the side stream; an epoch order computed in line
    on the engine stream (the first epoch, a cf_set_sampler_state jump, a new
    B) must be complete before that draw reads it.  The side-stream engine's
    batches equal the main-stream engine's, from a fresh engine and after a
    jump, on a graph big enough that the order takes a while."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine, synth_graph
    nu, ni = 200_000, 20_000
    ip, ix = synth_graph(nu, ni, 25.0, 0.8, 13, n_threads=8)
    B = 1 << 16
    out = []
    for side in (0, 1):
        e = Engine("bpr", nu, ni, 8, n_neg=1, seed=38)
        e.set_option("prep_stream", side)
        e.set_option("pipeline", 0)
        e.set_interactions(ip, ix)
        if jump:
            e.train_steps(B, 2)
            e.set_sampler_state(5, 7)
        got = [e.sample(B)[:2] for _ in range(3)]
        out.append(got)
        e.close()
    for b, ((p0, n0), (p1, n1)) in enumerate(zip(*out)):
        assert np.array_equal(p0, p1) and np.array_equal(n0, n1), b


def test_sorted_auto_falls_back_when_orders_do_not_fit(fold1):
    """Auto sorted batches need 2 x 16 B per pair for the two epoch orders;
    when HBM does not hold them beside the reserve (here: a reserve larger than
    any GPU), the engine keeps the unsorted batches -- the same batch sets --
    instead of failing with CF_ENOMEM, and cf_step_path reports it."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    B = 1000
    out = []
    for reserve in (1024, 1 << 30):
        e = Engine("bpr", nu, ni, 8, n_neg=1, seed=39)
        e.set_option("sorted_auto_reserve_mb", reserve)
        e.set_interactions(ip, ix)
        e.train_steps(B, 3)
        assert e.step_path(B)[1]["sorted_batches"] == (reserve == 1024), reserve
        out.append([e.sample(B)[0] for _ in range(4)])
        e.close()
    for b, (srt, plain) in enumerate(zip(*out)):
        ks = srt[:, 0].astype(np.int64) * ni + srt[:, 1]
        kp = plain[:, 0].astype(np.int64) * ni + plain[:, 1]
        assert (np.diff(ks) > 0).all() and not (np.diff(kp) > 0).all(), b
        assert np.array_equal(np.sort(kp), ks), b


@pytest.mark.parametrize("sb", [1, 3])
def test_sorted_batches_new_interactions_drop_cached_orders(fold1, sb):
    """A second cf_set_interactions (a smaller graph) must not reuse the
    epoch orders cached for the first: they index its larger pair array."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    e = Engine("bpr", nu, ni, 8, n_neg=1, seed=35)
    e.set_option("sorted_batches", sb)
    e.set_interactions(ip, ix)
    e.train_steps(100, 5)
    cut = 300   # users 0..299 keep their rows, the rest none
    ip2 = np.concatenate([ip[:cut + 1], np.full(nu - cut, ip[cut])]).astype(np.int64)
    ix2 = ix[:ip[cut]]
    e.set_interactions(ip2, ix2)
    e.train_steps(100, 5)
    for _ in range(len(ix2) // 100 + 2):   # across the new graph's epoch boundary
        pairs, _, _ = e.sample(100)
        assert (pairs[:, 0] < cut).all()
        assert all((ix2[ip2[u]:ip2[u + 1]] == i).any() for u, i in pairs[::7])
    e.close()


def test_negatives_uniform_over_complement(fold1):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    e = Engine("bpr", nu, ni, 1, n_neg=8, seed=6)
    e.set_interactions(ip, ix)
    counts = np.zeros(ni)
    expected = np.zeros(ni)
    deg = np.diff(ip)
    for _ in range(60):
        pairs, negs, _ = e.sample(4096)
        np.add.at(counts, negs.ravel(), 1)
        # each draw of user u is uniform over the n_items - deg(u) non-positives
        uc = np.bincount(pairs[:, 0], minlength=nu) * negs.shape[1]
        w = uc / (ni - deg)
        expected += w.sum()
        for u in np.nonzero(uc)[0]:
            expected[ix[ip[u]:ip[u + 1]]] -= w[u]
    chi2 = ((counts - expected) ** 2 / expected).sum()
    p = stats.chi2.sf(chi2, ni - 1)
    assert p > 1e-4, (chi2, p)
    e.close()


def test_gbpr_groups_are_item_positives(fold1):
    from collaborativefilteringusingtensorflow_amd.sampler_gbpr import Sampler
    R = make_csr_matrix(fold1)
    s = Sampler(R, gsize=3, n_neg=2, batch_size=100, seed=8)
    itemusers = csr_sets(*[np.asarray(a) for a in
                           (lambda c: (c.indptr, c.indices))(R.T.tocsr().sorted_indices())])
    counts = {}
    for _ in range(30):
        pairs, negs, groups = s.next_batch()
        assert groups.shape == (100, 3) and groups.dtype == np.int64
        for (u, i), g in zip(pairs, groups):
            for x in g:
                assert int(x) in itemusers[i]
    s.close()


def test_same_seed_same_stream(fold1):
    from collaborativefilteringusingtensorflow_amd.sampler_ranking import Sampler
    R = make_csr_matrix(fold1)
    a = Sampler(R, n_neg=3, batch_size=50, seed=99)
    b = Sampler(R, n_neg=3, batch_size=50, seed=99)
    c = Sampler(R, n_neg=3, batch_size=50, seed=100)
    for _ in range(5):
        pa, na = a.next_batch()
        pb, nb = b.next_batch()
        pc, nc = c.next_batch()
        assert np.array_equal(pa, pb) and np.array_equal(na, nb)
    assert not np.array_equal(pa, pc)
    for s in (a, b, c):
        s.close()


@pytest.mark.parametrize("model,W,G", [("bpr", 1, 1), ("bpr", 5, 1), ("bpr", 12, 1), ("gbpr", 5, 2)])
def test_pos_set_draw_equals_row_scan(fold1, model, W, G):
    """cf_set_option("neg_check"): the Pos(u) set probe and the CSR row scan
    take the same attempt sequence, so they draw identical batches -- on
    ml-100k fold 1 and on a dense toy graph where most candidates are
    rejected.  (neg_check 2, the one-lane-per-pair draw, exists only in a
    -DCF_LANE_DRAW build; it passed the same check at r02.)"""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    rng = np.random.RandomState(5)
    dense = []
    for u in range(30):   # 40 items, users own 5..38 of them
        dense.append(np.sort(rng.choice(40, size=rng.randint(5, 39), replace=False)).astype(np.int32))
    graphs = [(int(fold1["n_users"]), int(fold1["n_items"]), fold1["train_indptr"], fold1["train_indices"]),
              (30, 40, np.concatenate([[0], np.cumsum([len(r) for r in dense])]).astype(np.int64),
               np.concatenate(dense))]
    for gi, (nu, ni, ip, ix) in enumerate(graphs):
        out = []
        for check in (1, 0):
            e = Engine(model, nu, ni, 8, n_neg=W, gsize=G, seed=11)
            if gi == 0:   # set built by cf_set_interactions
                e.set_option("neg_check", check)
                e.set_interactions(ip, ix)
            else:         # set built when the option is selected
                e.set_interactions(ip, ix)
                e.set_option("neg_check", check)
            out.append([e.sample(64) for _ in range(12)])
            e.close()
        pos = csr_sets(ip, ix)
        for ba, bb in zip(*out):
            for xa, xb in zip(ba, bb):
                assert np.array_equal(xa, xb)
            pairs, negs = ba[0], ba[1]
            for (u, i), js in zip(pairs, negs):
                assert not any(int(j) in pos[u] for j in js)


def test_user_with_every_item_only_blocks_the_device_sampler():
    """A user whose row holds every item has no negative: the reference's
    rejection loop would spin forever (sampler_ranking.py:30-36) and the
    UITJ sampler skips such users (sampler_uitj_ranking.py:28).  The engine
    accepts the interactions; host-fed steps run, the device draw refuses."""
    from collaborativefilteringusingtensorflow_amd import _native as N
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    ni = 6
    ip = np.array([0, 6, 8, 9], dtype=np.int64)
    ix = np.array([0, 1, 2, 3, 4, 5, 1, 4, 2], dtype=np.int32)
    e = Engine("bpr", 3, ni, 8, n_neg=1, reg=0.05, seed=2)
    e.set_interactions(ip, ix)
    e.init_params(0.0, 0.1, seed=1)
    loss = e.step(np.array([[1, 1], [2, 2]], np.int32), np.array([[0], [5]], np.int32))
    assert np.isfinite(loss)
    with pytest.raises(N.NativeError, match="every item"):
        e.train_steps(2, 1)
    e.close()
