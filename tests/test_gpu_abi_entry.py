"""GPU checks of the SURVEY 8(b) entry points added in round 5: cf_train_epoch
(one iteration of the reference's train loop, bprmf.py:138-150), bitwise
against single steps each checked against the float64 oracle, and
cf_set_params / cf_get_params (every table in one call, NULL = keep)."""
import numpy as np
import pytest

from conftest import LocalStepCheck

pytestmark = pytest.mark.gpu


def _engine(fold1, seed=17, d=32, W=1, **kw):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    e = Engine("bpr", 943, 1682, d, n_neg=W, reg=0.05, seed=seed, **kw)
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    e.init_params(0.0, 0.1, truncated=True, seed=4)
    return e


TABLES = ("user", "item", "acc_user", "acc_item")


@pytest.mark.parametrize("B,W", [(4096, 1), (2048, 5)])
def test_train_epoch_matches_oracle_mean_loss(fold1, B, W):
    """cf_train_epoch = n_batches = int(nnz / B) device-sampled steps and the
    mean of their pre-update losses (the reference's TraLoss,
    bprmf.py:138-150).  In deterministic mode (order-free fixed-point sums)
    the epoch call is BITWISE the same model as n_batches single steps
    cf_train_steps(B, 1) of a second engine from the same state and sampler
    seed; each of those steps is checked against the float64 oracle from that
    engine's own pre-step tables, every element of every table within the
    a-priori fp32 bound (conftest.LocalStepCheck: a one-step bound is finite
    everywhere, so nothing goes unchecked), and the epoch's mean loss against
    the mean of the checked step losses."""
    nnz = int(fold1["train_indices"].shape[0])
    n_batches = nnz // B
    e = _engine(fold1, W=W)
    f = _engine(fold1, W=W)
    for x in (e, f):
        x.set_option("deterministic", 1)
    assert all(np.array_equal(e.get_table(t), f.get_table(t)) for t in TABLES)
    mean = e.train_epoch(B)
    assert e.sampler_state() in ((0, n_batches), (1, 0))   # ends at the epoch boundary
    chk = LocalStepCheck(0.05)
    losses = []
    for s in range(n_batches):
        st = f.sampler_state()
        pairs, negs, _ = f.sample(B)         # the batch the next step draws
        f.set_sampler_state(*st)
        chk.before(f)
        loss = f.train_steps(B, 1)
        chk.after(f, pairs, negs, loss, "step %d" % s)
        losses.append(loss)
    assert chk.excluded == 0
    for t in TABLES:
        assert np.array_equal(e.get_table(t), f.get_table(t)), t
    assert abs(mean - np.mean(losses)) <= 1e-12 * abs(np.mean(losses)), (mean, np.mean(losses))
    f.close()
    e.close()
    # (fast path) the next call is a whole epoch again; from inside an epoch, its rest
    e = _engine(fold1, W=W)
    e.train_epoch(B)
    e.train_epoch(B)
    e.train_steps(B, 3)
    e.profile_reset()
    e.profile(True)
    e.train_epoch(B)
    e.profile(False)
    steps = e.profile_read("apply_prep")[1] + e.profile_read("apply")[1]
    assert steps == n_batches - 3, (steps, n_batches)
    e.close()


def test_train_epoch_after_state_jump_on_fresh_engine(fold1):
    """cf_set_sampler_state(epoch, b > 0) on an engine that has not drawn yet:
    cf_train_epoch runs the epoch's remaining batches and stops at its end
    (the position is kept, as sampler_args keeps it)."""
    B = 4096
    n_batches = int(fold1["train_indices"].shape[0]) // B
    e = _engine(fold1)
    e.set_sampler_state(2, 4)
    e.profile_reset()
    e.profile(True)
    e.train_epoch(B)
    e.profile(False)
    steps = e.profile_read("apply_prep")[1] + e.profile_read("apply")[1]
    assert steps == n_batches - 4, (steps, n_batches)
    assert e.sampler_state() in ((2, n_batches), (3, 0))
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
