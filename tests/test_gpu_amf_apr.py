"""AMF apr mode (cf_config.amf_mode = CF_AMF_APR) on the GPU
against ``oracle.cf_oracle.amf_apr_step``, which tests/test_oracle.py pins
against torch autograd over the literal amf.py graph with __update_adv__'s
assigns run (amf.py:117-137, adv_method "grad").

Not a reference-parity mode: the reference computes Δ = 0 because those
assigns never run (SURVEY A.4 lists apr as the optional, non-parity mode).
Every step is checked step-locally: the oracle steps a float64 copy of the
engine's own pre-step tables, so fp32 drift of earlier steps does not widen
the band.  Tolerance: |gpu - oracle| <= 1e-6 + 1e-5 |oracle| elementwise
(conftest.assert_close) and the pre-update loss within 1e-5 relative.  Δ is a
normalised direction, so it carries the same relative error as the summed
gradient it comes from (fp32 float-atomic sums of <= a few hundred terms).
"""
import numpy as np
import pytest

from conftest import assert_close, get_stream
from oracle import cf_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5
TABLES = ("user", "item", "acc_user", "acc_item")
HP = dict(reg=0.05, reg_adv=1.0)


def _engine(fold1, d, W, eps=0.5, seed=51, **opts):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    e = Engine("amf", int(fold1["n_users"]), int(fold1["n_items"]), d, n_neg=W, seed=seed,
               epsilon=eps, amf_mode="apr", **HP)
    for k, v in opts.items():
        e.set_option(k, v)
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    e.init_params(0.0, 0.1, truncated=True, seed=4)
    return e


def _local_step(e, pairs, negs, eps):
    """One engine step against the oracle from the engine's own pre-step tables."""
    T = {t: e.get_table(t).astype(np.float64) for t in TABLES}
    lg = e.step(pairs, negs)
    lo = O.amf_apr_step(T["user"], T["item"], T["acc_user"], T["acc_item"], pairs, negs,
                        HP["reg"], eps, reg_adv=HP["reg_adv"])
    assert abs(lg - lo) <= RTOL * abs(lo), (lg, lo)
    for t in TABLES:
        assert_close(e.get_table(t), T[t], t)


@pytest.mark.parametrize("stream,d,opts", [
    ("rank_b100_w5", 40, {}),                     # apr_grad_kernel<EPL 4, W 5>
    ("rank_b100_w5", 128, {}),                    # EPL 8 (cfg5's width)
    ("rank_b100_w1", 64, {}),                     # W 1
    ("gbpr_b100_g3_w2", 24, {}),                  # runtime W (WT 0)
    ("rank_b100_w5", 40, {"slot_max": 1}),        # duplicated items past their slot: float atomics
    ("rank_b100_w5", 40, {"slot_max_user": 1}),   # users likewise
], ids=["w5-d40", "w5-d128", "w1-d64", "w2-d24", "item-atomics", "user-atomics"])
def test_apr_host_fed_steps_match_oracle(fold1, streams, stream, d, opts):
    """Phase 0 (plain BPR-form steps), the switch, then apr steps: a Δ row
    left in Gadv by one step would corrupt the next step's Δ."""
    st = get_stream(streams, stream)
    e = _engine(fold1, d, st["negs"].shape[2], **opts)
    for s in range(2):
        e.step(st["pairs"][s], st["negs"][s])
    e.begin_phase(1)
    for s in range(2, 14):
        _local_step(e, st["pairs"][s], st["negs"][s], 0.5)
    e.close()


def test_apr_epsilon_zero_is_reference_mode(fold1, streams):
    """epsilon = 0: Δ = 0, the apr kernels compute the reference mode's step."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    st = get_stream(streams, "rank_b100_w5")
    e = _engine(fold1, 32, 5, eps=0.0)
    e.begin_phase(1)
    for s in range(6):
        T = {t: e.get_table(t).astype(np.float64) for t in TABLES}
        lg = e.step(st["pairs"][s], st["negs"][s])
        lo = O.amf_step(T["user"], T["item"], T["acc_user"], T["acc_item"], st["pairs"][s],
                        st["negs"][s], HP["reg"], True, reg_adv=HP["reg_adv"])
        assert abs(lg - lo) <= RTOL * abs(lo), (s, lg, lo)
        for t in TABLES:
            assert_close(e.get_table(t), T[t], t)
    e.close()


@pytest.mark.parametrize("opts", [{}, {"pipeline": 0}, {"pipeline": 2}, {"prep_stream": 1, "pipeline": 0}],
                         ids=["pipelined", "stepwise", "draw-in-grad", "side-stream"])
def test_apr_train_steps_equals_host_fed_stream(fold1, opts):
    """cf_train_steps (device draw, pipelined) trains what cf_sample + cf_step
    train on the same sampler stream, in the apr phase."""
    K, B = 17, 100
    host = _engine(fold1, 40, 5)
    dev = _engine(fold1, 40, 5, **opts)
    host.begin_phase(1)
    dev.begin_phase(1)
    loss_h = 0.0
    for _ in range(K):
        pairs, negs, _g = host.sample(B)
        loss_h += host.step(pairs, negs)
    loss_d = dev.train_steps(B, K)
    assert abs(loss_d - loss_h) <= RTOL * abs(loss_h), (loss_d, loss_h)
    for t in TABLES:
        assert_close(dev.get_table(t), host.get_table(t), t)
    host.close()
    dev.close()


def test_apr_full_size_step():
    """cfg5's shape (1M users x 100K items, d = 128, W = 5, B = 65,536) in
    the apr phase: one step after three pipelined ones, against the oracle."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine, synth_graph
    nu, ni, d, W, B = 1_000_000, 100_000, 128, 5, 65536
    ip, ix = synth_graph(nu, ni, 50.0, 0.8, 20261015, n_threads=16)
    e = Engine("amf", nu, ni, d, n_neg=W, seed=78, epsilon=0.5, amf_mode="apr", **HP)
    e.set_interactions(ip, ix)
    del ip, ix
    e.init_params(0.0, 0.1, truncated=True, seed=1)
    e.begin_phase(1)
    e.train_steps(B, 3)
    pairs, negs, _g = e.sample(B)
    _local_step(e, pairs, negs, 0.5)
    e.close()


def test_apr_rejects_what_it_does_not_cover(fold1):
    from collaborativefilteringusingtensorflow_amd._native import NativeError
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    with pytest.raises(NativeError, match="AMF mode"):
        Engine("bpr", nu, ni, 16, amf_mode="apr")
    # multi-rank: the item sums cross ranks through a bound buffer, and the
    # gradient launch comes after the embed pass + the caller's all-reduce
    d = Engine("amf", nu, ni, 16, n_neg=5, amf_mode="apr", dense_item_apply=True)
    d.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    d.begin_phase(1)
    with pytest.raises(NativeError, match="bind the apr item buffer"):
        d.step_local_apr_embed(100)
    import torch
    buf = torch.zeros(ni * 16, dtype=torch.float32, device="cuda:0")
    d.bind_apr_item_grad(buf.data_ptr(), buf.numel())
    with pytest.raises(NativeError, match="cf_step_local_apr_embed and the all-reduce"):
        d.step_local_grad(100)
    d.close()
    e = _engine(fold1, 128, 5)
    with pytest.raises(NativeError, match="deterministic"):
        e.set_option("deterministic", 1)
    with pytest.raises(NativeError, match="item_slots"):
        e.set_option("item_slots", 1)
    e.close()


def test_amf_class_apr_trains(fold1):
    """The drop-in class with amf_mode="apr": a run through both phases trains
    (precision@10 well above random's ~0.01) and differs from the reference mode."""
    from collaborativefilteringusingtensorflow_amd.amf import AMF
    from collaborativefilteringusingtensorflow_amd import sampler_ranking
    from test_gpu_models import matrices
    tra, tst = matrices(fold1)
    m = ['pre', 'recall', 'map', 'mrr', 'ndcg']
    out = {}
    for mode in ("reference", "apr"):
        model = AMF(943, 1682, 10, 'cv', m, 1.0, 1.0, "grad", 0.05, 32, 100, max_iter=6, seed=9,
                    verbose=False, amf_mode=mode)
        sampler = sampler_ranking.Sampler(tra, n_neg=5, batch_size=100, seed=4)
        out[mode] = model.train(1, tra, tst, sampler)
        model.close()
        sampler.close()
        assert out[mode][0] > 0.05, (mode, out[mode])
    assert out["reference"] != out["apr"]


@pytest.mark.parametrize("B", [1, 17, 93])
def test_apr_ragged_batches(fold1, streams, B):
    """Batches that fill no block or wave evenly (the grid tails of the three
    apr launches), including a single pair whose rows are all seen once."""
    st = get_stream(streams, "rank_b100_w5")
    e = _engine(fold1, 72, 5)
    e.begin_phase(1)
    for s in range(4):
        _local_step(e, st["pairs"][s][:B], st["negs"][s][:B], 0.5)
    e.close()


def test_apr_hot_rows_in_one_batch(fold1):
    """One user and one positive in every pair of a batch, negatives drawn
    from a handful of items: every row is duplicated, user and positive
    past their slot caps (float atomics), Δ from the summed Gadv rows."""
    rng = np.random.RandomState(5)
    B, W = 96, 5
    pairs = np.stack([np.full(B, 7), np.full(B, 11)], 1).astype(np.int32)
    negs = rng.randint(100, 106, size=(B, W)).astype(np.int32)
    e = _engine(fold1, 40, W)
    e.begin_phase(1)
    for _ in range(3):
        _local_step(e, pairs, negs, 0.5)
    e.close()
