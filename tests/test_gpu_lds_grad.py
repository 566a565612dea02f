"""GPU parity of the gradient kernel with LDS-staged negative rows
(grad_lds_kernel: d = 128, W = 5; BPR, AMF, CML -- cfg3 / cfg5's
instantiation under grad_path 0) against the float64 oracle, on the
reference samplers' captured W = 5 batches over ml-100k fold 1.

Every path of the kernel's finish is covered: rows seen once (Adagrad in the
kernel), duplicated rows in slot rows or item records, hot rows past the slot
caps over every accumulator replica, the dense multi-rank item reduce,
deterministic mode, a ragged last block (B not a multiple of 16), and the
device-sampler pipeline (oracle replay of the drawn batches).  Reference semantics: bprmf.py:52-88,
amf.py:66-162, cml.py:55-129 (TF1 dedup-sum before SparseApplyAdagrad).

Tolerance: elementwise |gpu - oracle| <= 1e-6 + 1e-5 |oracle|
(conftest.assert_close), the per-step loss within 1e-5 relative; CML
trajectories CML_TRAJ (see test_gpu_bench_configs.py).
"""
import numpy as np
import pytest

from conftest import CML_TRAJ, assert_close, get_stream
from oracle import cf_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5
D = 128


def _engine(model, fold1, opts, **kw):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    e = Engine(model, int(fold1["n_users"]), int(fold1["n_items"]), D, n_neg=5,
               dense_item_apply=bool(opts.pop("dense", False)), seed=7, **kw)
    e.set_option("grad_path", opts.pop("grad_path", 3))
    for k, v in opts.items():
        e.set_option(k, v)
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    return e


def _tables(fold1, seed, truncated=True):
    rng = np.random.RandomState(seed)
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    return (O.init_table(rng, (nu, D), truncated=truncated),
            O.init_table(rng, (ni, D), truncated=truncated))


def _oracle(model, T, pairs, negs, adv, hp, n_items):
    if model == "bpr":
        return O.bpr_step(T["user"], T["item"], T["acc_user"], T["acc_item"], pairs, negs, hp["reg"])
    if model == "amf":
        return O.amf_step(T["user"], T["item"], T["acc_user"], T["acc_item"], pairs, negs, hp["reg"],
                          adv, reg_adv=hp["reg_adv"])
    return O.cml_step(T["user"], T["item"], T["acc_user"], T["acc_item"], pairs, negs,
                      hp["margin"], hp["reg_cov"], hp["clip_norm"],
                      use_rank_weight=hp.get("use_rank_weight", True), n_items=n_items)


HP = {"bpr": dict(reg=0.05), "amf": dict(reg=0.05, reg_adv=1.0),
      "cml": dict(margin=1.0, reg_cov=1.0, clip_norm=1.0)}


def _trajectory(fold1, stream, model, opts, K=30, switch=None, hp=None, B=None):
    hp = dict(HP[model] if hp is None else hp)
    U, V = _tables(fold1, 3, truncated=(model != "cml"))
    e = _engine(model, fold1, dict(opts), **hp)
    e.set_table("user", U)
    e.set_table("item", V)
    T = {"user": U.astype(np.float64), "item": V.astype(np.float64)}
    T["acc_user"] = np.full_like(T["user"], 0.1)
    T["acc_item"] = np.full_like(T["item"], 0.1)
    adv = False
    for s in range(K):
        if switch is not None and s == switch:
            e.begin_phase(1)
            adv = True
            T["acc_user"][...] = 0.1
            T["acc_item"][...] = 0.1
        pairs, negs = stream["pairs"][s], stream["negs"][s]
        if B is not None:
            pairs, negs = pairs[:B], negs[:B]
        lg = e.step(pairs, negs)
        lo = _oracle(model, T, pairs, negs, adv, hp, int(fold1["n_items"]))
        assert abs(lg - lo) <= RTOL * abs(lo) + (1e-6 if model == "cml" else 0.0), (s, lg, lo)
    tol = CML_TRAJ if model == "cml" else {}
    for t in ("user", "item", "acc_user", "acc_item"):
        assert_close(e.get_table(t), T[t], t, **tol)
    if model == "cml":
        for t in ("user", "item"):
            assert np.sqrt((e.get_table(t).astype(np.float64) ** 2).sum(1)).max() <= 1.0 + 1e-6
    e.close()


@pytest.mark.parametrize("item_slots", [0, 1], ids=["rows", "records"])
@pytest.mark.parametrize("model", ["bpr", "amf", "cml"])
def test_lds_kernel_trajectory(fold1, streams, model, item_slots):
    name = "rank_b50_w5" if model == "cml" else "rank_b100_w5"
    _trajectory(fold1, get_stream(streams, name), model, {"item_slots": item_slots},
                switch=15 if model == "amf" else None)


@pytest.mark.parametrize("reg_cov,use_rw", [(0.0, True), (0.5, False)])
def test_lds_kernel_cml_variants(fold1, streams, reg_cov, use_rw):
    hp = dict(margin=1.0, reg_cov=reg_cov, clip_norm=1.0, use_rank_weight=use_rw)
    _trajectory(fold1, get_stream(streams, "rank_b50_w5"), "cml", {}, hp=hp)


@pytest.mark.parametrize("slot_max,hot_replicas", [(1, 1), (2, 8), (256, 1)])
@pytest.mark.parametrize("item_slots", [0, 1], ids=["rows", "records"])
def test_lds_kernel_slot_regimes(fold1, streams, slot_max, hot_replicas, item_slots):
    """Duplicated rows split between slot store-and-sum and float atomics over
    hot_replicas accumulator copies; both user and item rows."""
    opts = {"slot_max": slot_max, "slot_max_user": slot_max, "hot_replicas": hot_replicas,
            "item_slots": item_slots}
    _trajectory(fold1, get_stream(streams, "rank_b100_w5"), "bpr", opts)


@pytest.mark.parametrize("opts", [{"item_reduce": 0}, {"item_reduce": 1}, {"item_reduce": 2}],
                         ids=["atomic", "reduce", "store-singletons"])
def test_lds_kernel_dense_items(fold1, streams, opts):
    """The multi-rank item path on one rank (dense item gradient + replicated
    item Adagrad): singleton item rows store their gradient row."""
    _trajectory(fold1, get_stream(streams, "rank_b100_w5"), "amf", dict(opts, dense=True), K=20)


def test_lds_kernel_deterministic(fold1, streams):
    _trajectory(fold1, get_stream(streams, "rank_b100_w5"), "bpr", {"deterministic": 1}, K=20)


@pytest.mark.parametrize("B", [1, 17, 93])
def test_lds_kernel_ragged_batch(fold1, streams, B):
    """Partial last blocks: groups past B stage nothing and store nothing."""
    _trajectory(fold1, get_stream(streams, "rank_b100_w5"), "amf", {}, K=12, B=B)


@pytest.mark.parametrize("model", ["amf", "cml"])
def test_lds_kernel_device_pipeline(fold1, model):
    """The device-sampler pipeline (cf_train_steps: the draw of step s+1 fused
    into the apply of step s) on the LDS kernel, replayed by the oracle on the
    identical batch stream (an engine with the same seed draws it with
    cf_sample).  CML at the shape its fp32-grounded band is pinned at
    (B = 100, 28 steps: tests/test_oracle.py::test_fp32_oracle_drift_bounds_cml_tolerance)."""
    B, K = (100, 28) if model == "cml" else (256, 20)
    dev = _engine(model, fold1, {}, **HP[model])
    rep = _engine(model, fold1, {}, **HP[model])
    for e in (dev, rep):
        e.init_params(0.0, 0.1, truncated=(model != "cml"), seed=6)
    T = {t: dev.get_table(t).astype(np.float64) for t in ("user", "item", "acc_user", "acc_item")}
    batches = [rep.sample(B) for _ in range(K)]
    rep.close()
    if model == "amf":
        dev.begin_phase(1)
    loss_dev = dev.train_steps(B, K)
    loss_ref = sum(_oracle(model, T, p, n, True, HP[model], int(fold1["n_items"])) for p, n, _ in batches)
    assert abs(loss_dev - loss_ref) <= RTOL * abs(loss_ref), (loss_dev, loss_ref)
    for t in T:
        assert_close(dev.get_table(t), T[t], t, **(CML_TRAJ if model == "cml" else {}))
    dev.close()


def test_lds_path_reported(fold1):
    """Auto (grad_path 0) takes the LDS-staged kernel at d = 128, W = 5."""
    for gp, want in ((0, True), (3, True), (2, False), (1, False)):
        e = _engine("amf", fold1, {"grad_path": gp}, **HP["amf"])
        flags, path = e.step_path(65536)
        assert path["lds"] == want, (gp, path)
        e.close()


@pytest.mark.parametrize("bias_slots", [0, 1], ids=["bias-atomics", "bias-slots"])
@pytest.mark.parametrize("item_slots", [0, 1], ids=["rows", "records"])
def test_lds_kernel_gbpr_d64(fold1, streams, item_slots, bias_slots):
    """GBPR (G = 1) on the LDS-staged kernel at d = 64 (grad_path 3; cfg4's
    shape): the reference's captured gbpr_b100_g1_w5 stream against the
    float64 oracle (gbprmf.py:58-106: V[j] without L2, b regularised)."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    st = get_stream(streams, "gbpr_b100_g1_w5")
    d, rho, reg = 64, 0.4, 0.01
    rng = np.random.RandomState(5)
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    U = O.init_table(rng, (nu, d))
    V = O.init_table(rng, (ni, d))
    b = O.init_table(rng, (ni,))
    e = Engine("gbpr", nu, ni, d, n_neg=5, gsize=1, rho=rho, reg=reg, seed=7)
    e.set_option("grad_path", 3)
    e.set_option("item_slots", item_slots)
    e.set_option("bias_slots", bias_slots)
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    e.set_table("user", U)
    e.set_table("item", V)
    e.set_table("bias", b)
    assert e.step_path(100)[1]["lds"]
    T = [U.astype(np.float64), V.astype(np.float64), b.astype(np.float64)]
    T += [np.full_like(T[0], 0.1), np.full_like(T[1], 0.1), np.full_like(T[2], 0.1)]
    for s in range(30):
        lg = e.step(st["pairs"][s], st["negs"][s], st["groups"][s])
        lo = O.gbpr_step(*T, st["pairs"][s], st["negs"][s], st["groups"][s], rho, reg)
        assert abs(lg - lo) <= RTOL * abs(lo), (s, lg, lo)
    for name, o in zip(("user", "item", "bias", "acc_user", "acc_item", "acc_bias"), T):
        assert_close(e.get_table(name), o, name)
    e.close()


@pytest.mark.parametrize("item_slots", [0, 1], ids=["rows", "records"])
@pytest.mark.parametrize("model,d", [("bpr", 32), ("amf", 128), ("cml", 128)])
def test_dense_rows_apply_pipeline(fold1, model, d, item_slots):
    """The dense item-row apply of the slot-row / record path (dense_apply 1,
    round 3: one group per item row instead of owners found among the
    occurrences; it engages when n_items <= 2 B (1 + W): here 1,682 items and
    B = 512, W = 5) in the device-sampler pipeline, replayed by the oracle on
    the identical batches; dense_apply 0 (the owner scan) lands on the same
    oracle.  CML takes 2 steps: at B = 512 its float32 oracle leaves the
    CML_TRAJ band around the float64 one by 2x after 6 steps (12.5x after
    12; 0.4-1.0x after 4, batch-dependent) and stays under 0.2 of it after 2
    (measured on the same kind of batches)."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    B, K = 512, (2 if model == "cml" else 12)
    hp = HP[model]
    for dense in (1, 0):
        def mk():
            e = Engine(model, int(fold1["n_users"]), int(fold1["n_items"]), d, n_neg=5, seed=7, **hp)
            e.set_option("item_slots", item_slots)
            e.set_option("dense_apply", dense)
            e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
            e.init_params(0.0, 0.1, truncated=(model != "cml"), seed=6)
            return e
        dev, rep = mk(), mk()
        T = {t: dev.get_table(t).astype(np.float64) for t in ("user", "item", "acc_user", "acc_item")}
        batches = [rep.sample(B) for _ in range(K)]
        rep.close()
        loss_dev = dev.train_steps(B, K)
        loss_ref = sum(_oracle(model, T, p_, n_, False, hp, int(fold1["n_items"])) for p_, n_, _ in batches)
        assert abs(loss_dev - loss_ref) <= RTOL * abs(loss_ref), (dense, loss_dev, loss_ref)
        for t in T:
            assert_close(dev.get_table(t), T[t], (t, dense), **(CML_TRAJ if model == "cml" else {}))
        dev.close()
