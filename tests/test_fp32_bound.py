"""The a-priori fp32 bound of oracle/fp32_bound.py (CPU).

The GPU parity tests of the BPR / AMF step compare every step of the engine
against the float64 oracle started from the engine's own pre-step tables,
elementwise within the bound E that forward error analysis gives for ANY
float32 implementation of the step (any summation order of the dedup-sum,
TF1's UnsortedSegmentSum before SparseApplyAdagrad, bprmf.py:83-88).

Here the bound itself is checked on the CPU:

* it holds for float32 implementations with different summation orders --
  the float32 oracle (np.add.at in occurrence order), the same with every
  row's occurrences shuffled, reversed, and summed as a pairwise tree, and
  the deterministic mode's fixed-point sums (2^-32 units);
* it is tight enough to catch an accumulation bug on a hot row: one
  occurrence dropped from, or added twice to, a row of 900 occurrences lands
  outside it.
"""
import numpy as np
import pytest

from conftest import get_stream
from oracle import cf_oracle as O
from oracle import fp32_bound as FB


def _dedup_f32(X, A, rows, grads, lr, order, rng):
    """dedup-sum + SparseApplyAdagrad in float32 with a chosen summation order
    per row: 'seq' (occurrence order), 'shuffle', 'reverse', 'tree'
    (pairwise), 'fx' (each term rounded to 2^-32, summed exactly, rounded
    once -- the deterministic mode)."""
    rows = np.asarray(rows).reshape(-1)
    g = np.asarray(grads, np.float32)
    uniq = np.unique(rows)
    G = np.zeros((uniq.shape[0], X.shape[1]), np.float32)
    by_row = {}
    for k, r in enumerate(rows.tolist()):
        by_row.setdefault(r, []).append(k)
    for q, r in enumerate(uniq.tolist()):
        ks = np.array(by_row[r])
        if order == "shuffle":
            ks = ks[rng.permutation(len(ks))]
        elif order == "reverse":
            ks = ks[::-1]
        terms = g[ks]
        if order == "tree":
            while terms.shape[0] > 1:
                if terms.shape[0] % 2:
                    terms = np.concatenate([terms, np.zeros_like(terms[:1])])
                terms = (terms[0::2] + terms[1::2]).astype(np.float32)
            G[q] = terms[0]
        elif order == "fx":
            fx = np.rint(terms.astype(np.float64) * 2.0 ** 32).astype(np.int64)
            G[q] = (fx.sum(axis=0).astype(np.float64) * 2.0 ** -32).astype(np.float32)
        else:
            acc = np.zeros(X.shape[1], np.float32)
            for t in terms:
                acc = (acc + t).astype(np.float32)
            G[q] = acc
    A[uniq] += G * G
    X[uniq] -= (np.float32(lr) * G) / np.sqrt(A[uniq])


def f32_step(T, pairs, negs, reg, order, rng, adversarial=None):
    """One BPR (or AMF) step in float32 with the given dedup order."""
    U, V, AU, AV = T
    c_scale = None
    if adversarial:
        Uu, Vi, Vj = U[pairs[:, 0]], V[pairs[:, 1]], V[negs]
        x = np.sum(Uu * Vi, axis=1)[:, None] - np.sum(Uu[:, None, :] * Vj, axis=-1)
        c_scale = (np.float32(1) + np.float32(1.0) * ((x >= -80) & (x <= 1e8))).astype(np.float32)
    _, _, (ur, ug), (vr, vg) = O.bpr_loss_grads(U, V, pairs, negs, reg, c_scale)
    _dedup_f32(U, AU, ur, ug, 0.1, order, rng)
    _dedup_f32(V, AV, vr, vg, 0.1, order, rng)


def local_worst(T32_before, T32_after, pairs, negs, reg, adversarial=None):
    """max over elements of |f32 - f64| / E for one step from T32_before."""
    L = [t.astype(np.float64) for t in T32_before]
    E = FB.zero_bounds(L[0], L[1], acc_exact=True)
    FB.bpr_step_bounded(*L, E, pairs, negs, reg, adversarial=adversarial)
    worst = 0.0
    for q, k in enumerate(FB.TABLES):
        err = np.abs(T32_after[q].astype(np.float64) - L[q])
        assert np.all(err[E[k] == 0] == 0), k        # untouched rows are bit-identical
        nz = E[k] > 0
        if nz.any():
            worst = max(worst, float((err[nz] / E[k][nz]).max()))
    return worst


def hot_batches(rng, n_users=400, n_items=300, B=1200, hot=7, n_hot=900, K=3, W=1):
    """Batches whose item `hot` is the positive of n_hot pairs (600) and the
    negative of the rest (300): the shape of test_pos_sort_hot_item."""
    out = []
    for _ in range(K):
        u = rng.randint(n_users, size=B).astype(np.int32)
        i = rng.randint(n_items, size=B).astype(np.int32)
        i[:600] = hot
        j = rng.randint(n_items, size=(B, W)).astype(np.int32)
        j[600:n_hot, 0] = hot
        out.append((np.stack([u, i], 1), j))
    return out


def tabs(rng, nu, ni, d):
    return [O.init_table(rng, (nu, d)), O.init_table(rng, (ni, d)),
            np.full((nu, d), 0.1, np.float32), np.full((ni, d), 0.1, np.float32)]


@pytest.mark.parametrize("order", ["seq", "shuffle", "reverse", "tree", "fx"])
@pytest.mark.parametrize("name,d,reg", [("rank_b100_w1", 32, 0.1), ("rank_b100_w5", 64, 0.05),
                                        ("uij_b100", 16, 0.02)])
def test_bound_holds_for_every_order_on_reference_streams(streams, name, d, reg, order):
    st = get_stream(streams, name)
    rng = np.random.RandomState(3)
    T = tabs(rng, 943, 1682, d)
    worst = 0.0
    for s in range(12):
        before = [t.copy() for t in T]
        f32_step(T, st["pairs"][s], st["negs"][s], reg, order, rng)
        worst = max(worst, local_worst(before, T, st["pairs"][s], st["negs"][s], reg))
    assert worst <= 1.0, worst


@pytest.mark.parametrize("order", ["seq", "shuffle", "reverse", "tree", "fx"])
@pytest.mark.parametrize("adversarial", [None, True])
def test_bound_holds_on_hot_rows(order, adversarial):
    rng = np.random.RandomState(11)
    T = tabs(rng, 400, 300, 16)
    worst = 0.0
    for pairs, negs in hot_batches(rng):
        before = [t.copy() for t in T]
        f32_step(T, pairs, negs, 0.02, order, rng, adversarial)
        worst = max(worst, local_worst(before, T, pairs, negs, 0.02, adversarial))
    assert worst <= 1.0, worst


@pytest.mark.parametrize("bug", ["drop", "twice"])
def test_bound_catches_one_occurrence_on_a_hot_row(bug):
    """One of the hot item's 900 occurrences dropped from its sum (or added
    twice): its row leaves the bound on every step."""
    rng = np.random.RandomState(5)
    T = tabs(rng, 400, 300, 16)
    for pairs, negs in hot_batches(rng):
        before = [t.copy() for t in T]
        U, V, AU, AV = T
        _, _, (ur, ug), (vr, vg) = O.bpr_loss_grads(U, V, pairs, negs, 0.02)
        k = int(np.nonzero(vr == 7)[0][rng.randint(900)])
        if bug == "drop":
            vr, vg = np.delete(vr, k), np.delete(vg, k, axis=0)
        else:
            vr, vg = np.append(vr, vr[k]), np.concatenate([vg, vg[k:k + 1]])
        _dedup_f32(U, AU, ur, ug, 0.1, "seq", rng)
        _dedup_f32(V, AV, vr, vg, 0.1, "seq", rng)
        L = [t.astype(np.float64) for t in before]
        E = FB.zero_bounds(L[0], L[1], acc_exact=True)
        FB.bpr_step_bounded(*L, E, pairs, negs, 0.02)
        ratio = np.abs(V[7].astype(np.float64) - L[1][7]) / E["item"][7]
        assert ratio.max() > 3.0, ratio.max()
        # every other item row stays inside
        rest = np.delete(np.arange(300), 7)
        assert (np.abs(V[rest].astype(np.float64) - L[1][rest]) <= E["item"][rest]).all()
        T = [U, V, AU, AV]


def test_forward_bound_covers_fp32_trajectory(streams):
    """Carried over steps (tables within E of the float64 ones), the bound
    still holds for the float32 oracle's whole trajectory."""
    st = get_stream(streams, "rank_b100_w1")
    rng = np.random.RandomState(3)
    T = tabs(rng, 943, 1682, 32)
    L = [t.astype(np.float64) for t in T]
    L[2][...] = 0.1
    L[3][...] = 0.1
    E = FB.zero_bounds(L[0], L[1])
    for s in range(20):
        f32_step(T, st["pairs"][s], st["negs"][s], 0.1, "seq", rng)
        FB.bpr_step_bounded(*L, E, st["pairs"][s], st["negs"][s], 0.1)
        for q, k in enumerate(FB.TABLES):
            assert (np.abs(T[q].astype(np.float64) - L[q]) <= E[k]).all(), (s, k)


def _cml_local(before, after, pairs, negs, **hp):
    L = [t.astype(np.float64) for t in before]
    E = FB.zero_bounds(L[0], L[1], acc_exact=True)
    FB.cml_step_bounded(*L, E, pairs, negs, **hp)
    worst, excluded = 0.0, 0
    for q, k in enumerate(FB.TABLES):
        err = np.abs(after[q].astype(np.float64) - L[q])
        fin = np.isfinite(E[k])
        excluded += int((~fin).any(axis=1).sum())
        assert np.all(err[fin & (E[k] == 0)] == 0), k
        nz = fin & (E[k] > 0)
        if nz.any():
            worst = max(worst, float((err[nz] / E[k][nz]).max()))
    return worst, excluded, L, E


CML_HP = dict(margin=1.0, reg_cov=1.0, clip_norm=1.0, use_rank_weight=True)


@pytest.mark.parametrize("name,d", [("rank_b50_w5", 50), ("rank_b100_w5", 128)])
def test_cml_bound_holds_on_reference_streams(streams, name, d):
    """The float32 oracle's CML steps (hinge, rank weight, argmin, clip of
    every row) stay inside the local bound, and no pair is near a branch."""
    st = get_stream(streams, name)
    rng = np.random.RandomState(3)
    T = [O.init_table(rng, (943, d), truncated=False), O.init_table(rng, (1682, d), truncated=False),
         np.full((943, d), 0.1, np.float32), np.full((1682, d), 0.1, np.float32)]
    worst = 0.0
    for s in range(20):
        before = [t.copy() for t in T]
        O.cml_step(*T, st["pairs"][s], st["negs"][s], **CML_HP)
        w, excluded, _, _ = _cml_local(before, T, st["pairs"][s], st["negs"][s], **CML_HP)
        assert excluded == 0
        worst = max(worst, w)
    assert worst <= 1.0, worst


def test_cml_bound_catches_one_occurrence_on_a_hot_row():
    """A CML item negative in 300 pairs: one of its occurrences dropped from
    the dedup-sum lands outside the bound."""
    rng = np.random.RandomState(8)
    nu, ni, d, B, W = 400, 300, 16, 600, 5
    T = [O.init_table(rng, (nu, d), truncated=False), O.init_table(rng, (ni, d), truncated=False),
         np.full((nu, d), 0.1, np.float32), np.full((ni, d), 0.1, np.float32)]
    pairs = np.stack([rng.randint(nu, size=B), rng.randint(ni, size=B)], 1).astype(np.int32)
    negs = rng.randint(ni, size=(B, W)).astype(np.int32)
    negs[:300, 0] = 7
    before = [t.copy() for t in T]
    # the float32 step with one occurrence of item 7 missing from its sum
    U, V, AU, AV = T
    keep = np.ones(B, dtype=bool)
    keep[int(rng.randint(300))] = False
    L32 = [t.copy() for t in before]
    O.cml_step(*L32, pairs, negs, **CML_HP)                       # the correct float32 step
    T2 = [t.copy() for t in before]
    O.cml_step(*T2, pairs[keep], negs[keep], **CML_HP)            # item 7 loses one occurrence
    w_ok, _, L, E = _cml_local(before, L32, pairs, negs, **CML_HP)
    assert w_ok <= 1.0
    # the row itself barely moves (Adagrad's first step is ~lr * sign(G) for a
    # large summed G, then the clip), its accumulator G^2 does
    ratio = np.abs(T2[3][7].astype(np.float64) - L[3][7]) / E["acc_item"][7]
    assert ratio.max() > 3.0, ratio.max()


def _fold_batches(fold1, rng, B, W, n):
    """Uniform pairs of ml-100k fold 1 with W negatives outside Pos(u)."""
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    users = np.repeat(np.arange(len(ip) - 1), np.diff(ip))
    out = []
    for _ in range(n):
        q = rng.choice(len(ix), B, replace=False)
        negs = rng.randint(0, 1682, (B, W))
        for r in range(B):
            row = ix[ip[users[q[r]]]:ip[users[q[r]] + 1]]
            while np.isin(negs[r], row).any():
                negs[r] = rng.randint(0, 1682, W)
        out.append((np.stack([users[q], ix[q]], 1).astype(np.int32), negs.astype(np.int32)))
    return out


def test_carried_bound_goes_inf_never_nan(fold1):
    """The shape of round 5's cf_train_epoch trajectory check (d = 32,
    B = 2048, W = 5, 21 steps): the bound carried over the epoch outgrows the
    Zipf head's accumulators and reads inf on most elements.  It must never
    read NaN (which compares false with everything, and raised a
    RuntimeWarning), and conftest.assert_close must refuse to pass the
    unbounded elements silently -- it fails unless the caller allows and
    counts them (max_excluded)."""
    import warnings
    from conftest import assert_close
    rng = np.random.RandomState(9)
    T = [t.astype(np.float64) for t in tabs(rng, 943, 1682, 32)]
    E = FB.zero_bounds(T[0], T[1], acc_exact=True)
    with warnings.catch_warnings():
        warnings.simplefilter("error")   # a RuntimeWarning from the bound fails the test
        for pairs, negs in _fold_batches(fold1, rng, 2048, 5, 21):
            FB.bpr_step_bounded(*T, E, pairs, negs, 0.05)
    assert not any(np.isnan(E[k]).any() for k in FB.TABLES)
    frac = (~np.isfinite(E["item"])).mean()
    assert frac > 0.5, frac               # the carried bound checks (almost) nothing here
    with pytest.raises(AssertionError, match="non-finite a-priori bound"):
        assert_close(T[1], T[1], "item", bound=E["item"])
    with pytest.raises(AssertionError, match="non-finite a-priori bound"):
        assert_close(T[1], T[1], "item", bound=E["item"], max_excluded=0.01)
    assert_close(T[1], T[1], "item", bound=E["item"], max_excluded=1.0)   # allowed and counted


def test_one_step_bound_is_finite_everywhere(fold1):
    """The per-step check (conftest.LocalStepCheck) needs a finite E on every
    element: one step from any tables, at that same shape, gives one."""
    rng = np.random.RandomState(10)
    T = [t.astype(np.float64) for t in tabs(rng, 943, 1682, 32)]
    batches = _fold_batches(fold1, rng, 2048, 5, 6)
    for pairs, negs in batches:
        O.bpr_step(*T, pairs, negs, 0.05)          # move the tables off their init
    for pairs, negs in batches[:2]:
        E = FB.zero_bounds(T[0], T[1], acc_exact=True)
        FB.bpr_step_bounded(*[t.copy() for t in T], E, pairs, negs, 0.05)
        assert all(np.isfinite(E[k]).all() for k in FB.TABLES)
