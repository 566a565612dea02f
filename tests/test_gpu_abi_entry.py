"""GPU checks of the SURVEY 8(b) entry points added in round 5: cf_train_epoch
(one iteration of the reference's train loop, bprmf.py:138-150) against the
float64 oracle's epoch mean loss on the identical batch stream, and
cf_set_params / cf_get_params (every table in one call, NULL = keep)."""
import numpy as np
import pytest

from conftest import assert_close
from oracle import cf_oracle as O

pytestmark = pytest.mark.gpu


def _engine(fold1, seed=17, d=32, W=1, **kw):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    e = Engine("bpr", 943, 1682, d, n_neg=W, reg=0.05, seed=seed, **kw)
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    e.init_params(0.0, 0.1, truncated=True, seed=4)
    return e


@pytest.mark.parametrize("B,W", [(4096, 1), (2048, 5)])
def test_train_epoch_matches_oracle_mean_loss(fold1, B, W):
    """cf_train_epoch = n_batches = int(nnz / B) device-sampled steps and the
    mean of their pre-update losses (the reference's TraLoss).  A second
    engine with the same seed draws the same stream with cf_sample; the
    float64 oracle steps those batches from the same initial tables.  The
    tables after the epoch are checked in the strict band plus the a-priori
    fp32 bound carried over the epoch (oracle/fp32_bound.py: ml-100k's head
    items sum hundreds of occurrences per step)."""
    from oracle import fp32_bound as FB
    nnz = int(fold1["train_indices"].shape[0])
    n_batches = nnz // B
    e = _engine(fold1, W=W)
    T0 = {t: e.get_table(t).astype(np.float64) for t in ("user", "item", "acc_user", "acc_item")}
    mean = e.train_epoch(B)
    assert e.sampler_state() in ((0, n_batches), (1, 0))   # ends at the epoch boundary
    f = _engine(fold1, W=W)
    batches = [f.sample(B)[:2] for _ in range(n_batches)]
    f.close()
    U, V, AU, AV = T0["user"], T0["item"], T0["acc_user"], T0["acc_item"]
    E = FB.zero_bounds(U, V, acc_exact=True)
    losses = [FB.bpr_step_bounded(U, V, AU, AV, E, p, n, 0.05) for p, n in batches]
    assert abs(mean - np.mean(losses)) <= 1e-5 * abs(np.mean(losses)), (mean, np.mean(losses))
    for t, o in (("user", U), ("item", V), ("acc_user", AU), ("acc_item", AV)):
        assert_close(e.get_table(t), o, t, bound=E[t])
    # the next call is a whole epoch again; from inside an epoch, its rest
    e.train_epoch(B)
    e.train_steps(B, 3)
    ep, bt = e.sampler_state()
    e.profile_reset()
    e.profile(True)
    e.train_epoch(B)
    e.profile(False)
    steps = e.profile_read("apply_prep")[1] + e.profile_read("apply")[1]
    assert steps == n_batches - 3, (steps, n_batches)
    e.close()


def test_set_get_params_roundtrip(fold1):
    """All tables in one call; NULL keeps a table; b / Ab only on the bias
    models; a bad argument copies nothing."""
    from collaborativefilteringusingtensorflow_amd import _native as N
    e = _engine(fold1)
    rng = np.random.RandomState(3)
    T = {"user": rng.rand(943, 32), "item": rng.rand(1682, 32), "acc_user": rng.rand(943, 32) + 0.1,
         "acc_item": rng.rand(1682, 32) + 0.1}
    T = {k: v.astype(np.float32) for k, v in T.items()}
    e.set_params(**T)
    got = e.get_params()
    assert sorted(got) == sorted(T)
    for k in T:
        assert np.array_equal(got[k], T[k]), k
    U2 = (T["user"] * 2).astype(np.float32)
    e.set_params(user=U2)                     # the rest kept
    got = e.get_params(["user", "item"])
    assert np.array_equal(got["user"], U2) and np.array_equal(got["item"], T["item"])
    with pytest.raises(N.NativeError, match="not present"):
        e.set_params(user=T["user"], bias=np.zeros(1682, np.float32))
    assert np.array_equal(e.get_table("user"), U2)   # nothing copied
    e.close()
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    g = Engine("gbpr", 943, 1682, 16, n_neg=1, gsize=1, seed=2)
    b = rng.rand(1682).astype(np.float32)
    g.set_params(bias=b, acc_bias=b + 1)
    got = g.get_params()
    assert np.array_equal(got["bias"], b) and np.array_equal(got["acc_bias"], b + 1)
    g.close()
