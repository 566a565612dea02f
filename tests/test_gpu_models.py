"""End-to-end GPU tests of the drop-in model classes, and full-size parity.

* cfg1 (BASELINE configs[0]): BPRMF on ml-100k fold 1, d=32, the testbprmf.py
  hyper-parameters (reg=.1, B=100, W=1, topN=10, 50 epochs), fed the
  reference sampler's own stream for np.random.seed(11) (bit-exact host
  sampler) and the same initial tables as the CPU oracle (oracle/cf_oracle.c,
  fp32): ranking metrics after training must agree within 0.2 % (north star).
* the same drivers' device-sampled path trains (metrics far above random).
* cfg2 at full size (1M users x 100K items, d=64): one step at B=65,536 on a
  device-drawn batch, and two pipelined steps at the bench batch B=2^19
  (pos_sort, partials past capP on atomics) against the float64 oracle,
  elementwise |gpu - oracle| <= 1e-6 + 1e-5 |oracle| over the whole tables.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import assert_close
from oracle import cf_oracle as O

pytestmark = pytest.mark.gpu


class ListSampler(object):
    """A plain host sampler (like the reference's thread sampler)."""

    def __init__(self, batches):
        self._it = iter(batches)

    def next_batch(self):
        return next(self._it)


def matrices(fold1):
    nu, ni = int(fold1["n_users"]), int(fold1["n_items"])
    tra = sp.csr_matrix((np.ones(len(fold1["train_indices"]), np.float32),
                         fold1["train_indices"], fold1["train_indptr"]), shape=(nu, ni))
    tst = sp.csr_matrix((np.ones(len(fold1["test_indices"]), np.float32),
                         fold1["test_indices"], fold1["test_indptr"]), shape=(nu, ni))
    return sp.lil_matrix(tra), sp.lil_matrix(tst)


def oracle_metrics(U, V, fold1, topN, metrics):
    from collaborativefilteringusingtensorflow_amd.ranking import evaluateCV
    tst_ip, tst_ix = fold1["test_indptr"], fold1["test_indices"]
    users = list(set(np.nonzero(np.diff(tst_ip))[0].tolist()))
    yt = [set(tst_ix[tst_ip[u]:tst_ip[u + 1]].tolist()) for u in users]
    S = O.predict("bpr", U.astype(np.float64), V.astype(np.float64), None, users)
    yp = O.recommend(S, fold1["train_indptr"], fold1["train_indices"], users, topN)
    return evaluateCV(yt, yp, metrics, topN)


@pytest.mark.parametrize("epochs", [50])
def test_cfg1_bprmf_metrics_match_oracle(fold1, epochs):
    from collaborativefilteringusingtensorflow_amd.bprmf import BPRMF
    from oracle.build_oracle import COracle
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    B, d, reg, topN = 100, 32, 0.1, 10
    metrics = ['pre', 'recall', 'map', 'mrr', 'ndcg']
    n_batches = len(ix) // B
    # the reference's own sampler stream for np.random.seed(11) (bit-exact
    # host mode, pinned to the captured reference batches in test_exact_sampler)
    from collaborativefilteringusingtensorflow_amd.sampler_ranking import ExactSampler
    tra, tst = matrices(fold1)
    es = ExactSampler(tra, n_neg=1, batch_size=B, seed=11)
    batches = [es.next_batch() for _ in range(n_batches * epochs)]
    es.close()
    init_rng = np.random.RandomState(11)
    U0 = O.init_table(init_rng, (943, d))
    V0 = O.init_table(init_rng, (1682, d))

    # CPU oracle (fp32 C restatement), identical batches and init
    c = COracle("bpr", U0, V0, W=1, reg=reg)
    for pairs, negs in batches:
        c.step(pairs, negs)
    ref = oracle_metrics(c.U, c.V, fold1, topN, metrics)

    # GPU: the drop-in model class fed by the exact sampler itself
    model = BPRMF(943, 1682, topN, 'cv', metrics, reg, d, B, max_iter=epochs, seed=5,
                  verbose=False)
    model.set_initial_tables(user=U0, item=V0)
    got = model.train(1, tra, tst, ExactSampler(tra, n_neg=1, batch_size=B, seed=11))
    drift_u = np.abs(model.engine.get_table("user") - c.U).max() / np.abs(c.U).max()
    model.close()
    print("oracle", ref, "gpu", got, "table drift", drift_u)
    for m, a, b in zip(metrics, got, ref):
        assert abs(a - b) <= 2e-3 * abs(b), (m, a, b)
    assert ref[metrics.index('ndcg')] > 0.2   # trained, not random
    # the committed cfg1 golden (tests/golden/make_cfg1_golden.py) is this
    # same oracle run: bench.py reports NDCG@10 against it
    import json, os
    with open(os.path.join(os.path.dirname(__file__), "golden", "cfg1_oracle_metrics.json")) as f:
        g = json.load(f)["metrics"]
    for m, b in zip(metrics, ref):
        assert abs(g[m] - b) <= 1e-9 * abs(b), (m, g[m], b)


def test_device_sampled_drivers_train(fold1):
    from collaborativefilteringusingtensorflow_amd.bprmf import BPRMF
    from collaborativefilteringusingtensorflow_amd.gbprmf import GBPRMF
    from collaborativefilteringusingtensorflow_amd.cml import CML
    from collaborativefilteringusingtensorflow_amd.amf import AMF
    from collaborativefilteringusingtensorflow_amd import sampler_ranking, sampler_gbpr
    tra, tst = matrices(fold1)
    m = ['pre', 'recall', 'map', 'mrr', 'ndcg']
    runs = [
        (BPRMF(943, 1682, 10, 'cv', m, 0.1, 32, 100, max_iter=6, verbose=False),
         sampler_ranking.Sampler(tra, n_neg=1, batch_size=100, seed=1)),
        (GBPRMF(943, 1682, 10, 0.4, 1, 'cv', m, 0.01, 32, 100, max_iter=6, verbose=False),
         sampler_gbpr.Sampler(tra, 1, 5, 100, seed=2)),
        (CML(943, 1682, 10, 'cv', m, 1.0, 1.0, True, 1.0, 50, 50, max_iter=4, verbose=False),
         sampler_ranking.Sampler(tra, n_neg=5, batch_size=50, seed=3)),
        (AMF(943, 1682, 10, 'cv', m, 1.0, 1.0, "grad", 0.05, 32, 100, max_iter=6,
             verbose=False),
         sampler_ranking.Sampler(tra, n_neg=5, batch_size=100, seed=4)),
    ]
    for model, sampler in runs:
        scores = model.train(1, tra, tst, sampler)
        assert len(scores) == 5
        if isinstance(model, CML):
            # CML returns the topN=1000 scores (cml.py:203-212): recall@1000
            assert scores[1] > 0.5, scores
        else:
            # random recommendation on ml-100k gives precision@10 ~ 0.01
            assert scores[0] > 0.05, (type(model).__name__, scores)
        st = sampler.state()
        assert st[0] >= 3  # the sampler stream advanced with training
        model.close()
        sampler.close()


def test_amf_rejects_rand():
    from collaborativefilteringusingtensorflow_amd.amf import AMF
    with pytest.raises(ValueError):
        AMF(10, 10, adv_method="rand")


@pytest.fixture(scope="module")
def cfg2_graph():
    from collaborativefilteringusingtensorflow_amd.engine import synth_graph
    return synth_graph(1_000_000, 100_000, 50.0, 0.8, 20261015, n_threads=16)


def test_cfg2_full_size_step_parity(cfg2_graph):
    """cfg2 at SURVEY 8(d)'s B = 65,536 (pos_sort auto: off): one host-fed
    step on a device-drawn batch against the float64 oracle, elementwise."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni, d, B = 1_000_000, 100_000, 64, 65536
    ip, ix = cfg2_graph
    e = Engine("bpr", nu, ni, d, n_neg=1, reg=0.02, seed=77)
    e.set_interactions(ip, ix)
    e.init_params(0.0, 0.1, truncated=True, seed=1)
    e.train_steps(B, 3)                      # move off the initial state
    U = e.get_table("user").astype(np.float64)
    V = e.get_table("item").astype(np.float64)
    AU = e.get_table("acc_user").astype(np.float64)
    AV = e.get_table("acc_item").astype(np.float64)
    pairs, negs, _ = e.sample(B)
    # sampler invariants at full size (sorted CSR row membership)
    k = pairs[:, 0].astype(np.int64)
    rows_lo, rows_hi = ip[k], ip[k + 1]
    for r in np.random.RandomState(0).choice(B, 2000, replace=False):
        row = ix[rows_lo[r]:rows_hi[r]]
        assert pairs[r, 1] in row and negs[r, 0] not in row
    loss = e.step(pairs, negs)
    lo = O.bpr_step(U, V, AU, AV, pairs, negs, 0.02)
    assert abs(loss - lo) <= 1e-5 * abs(lo)
    for name, ref in (("user", U), ("item", V), ("acc_user", AU), ("acc_item", AV)):
        assert_close(e.get_table(name), ref, name)
    e.close()


def test_cfg2_bench_batch_pos_sort_matches_oracle(cfg2_graph):
    """The benched cfg2 instantiation itself: B = 2^19 pairs per step with
    pos_sort auto (on), i.e. psort + grad_sort_kernel<BPR, d 64, W 1> + the
    pos_sort apply fused with the next draw (apply_ps_kernel), where the
    Zipf-head positives' partials overflow capP into float atomics.  Three
    pipelined steps move off the initial state; then two more pipelined
    steps (cf_train_steps: the first one's apply launch draws the second's
    batch) are replayed by the float64 oracle on the same drawn batches and
    compared over the WHOLE tables, elementwise (bprmf.py:83-88: TF1's
    dedup-sum before SparseApplyAdagrad)."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni, d, B, K, reg = 1_000_000, 100_000, 64, 1 << 19, 2, 0.02
    ip, ix = cfg2_graph
    e = Engine("bpr", nu, ni, d, n_neg=1, reg=reg, seed=78)
    e.set_interactions(ip, ix)
    e.init_params(0.0, 0.1, truncated=True, seed=1)
    e.profile_reset()
    e.profile(True)
    e.train_steps(B, 3)
    T = {t: e.get_table(t).astype(np.float64) for t in ("user", "item", "acc_user", "acc_item")}
    st = e.sampler_state()
    batches = [e.sample(B)[:2] for _ in range(K)]
    e.set_sampler_state(*st)
    loss = e.train_steps(B, K)
    e.profile(False)
    assert e.profile_read("psort")[1] == 3 + K, "pos_sort did not run at the bench batch"
    # the drawn batches overflow the positives' partial slots (capP = 8):
    # partial k of item i covers sorted positions of block offP[i] / 16 + k
    for pairs, _ in batches:
        cnt = np.bincount(pairs[:, 1], minlength=ni)
        off = np.cumsum(cnt) - cnt
        nparts = np.where(cnt > 0, (off + cnt - 1) // 16 - off // 16 + 1, 0)
        assert (nparts > 8).sum() > 100, int((nparts > 8).sum())
    lo = 0.0
    for pairs, negs in batches:
        lo += O.bpr_step(T["user"], T["item"], T["acc_user"], T["acc_item"], pairs, negs, reg)
    assert abs(loss - lo) <= 1e-5 * abs(lo), (loss, lo)
    for t in T:
        assert_close(e.get_table(t), T[t], t)
    e.close()


def _dev_used():
    from collaborativefilteringusingtensorflow_amd import _native as N   # noqa: F401 (one HIP runtime)
    import torch
    torch.cuda.synchronize()
    free, total = torch.cuda.mem_get_info(0)
    return total - free


def test_cfg2_deterministic_memory(cfg2_graph):
    """Deterministic mode at the benched cfg2 instantiation (B = 2^19,
    pos_sort, fixed point) allocates its users-past-their-cap rows compactly
    (one int64 row per hot user of the batch, at most B / (capU + 1), found
    by psort) instead of a dense [n_users, d] int64 array (512 MB at cfg2;
    round-4 verdict item 8).  Device memory of a deterministic engine after
    two steps, less that of the fast engine, measured with hipMemGetInfo:
    was ~630 MB (GU64 512 + GV64 51 + slotP64 68), now under 250 MB."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    nu, ni, d, B = 1_000_000, 100_000, 64, 1 << 19
    ip, ix = cfg2_graph
    used = {}
    for det in (0, 1):
        base = _dev_used()
        e = Engine("bpr", nu, ni, d, n_neg=1, reg=0.02, seed=78)
        e.set_option("deterministic", det)
        e.set_interactions(ip, ix)
        e.init_params(0.0, 0.1, truncated=True, seed=1)
        loss = e.train_steps(B, 2)
        assert np.isfinite(loss)
        used[det] = _dev_used() - base
        assert e.step_path(B)[1]["deterministic"] == bool(det)
        e.close()
    extra = (used[1] - used[0]) / 2 ** 20
    print("deterministic extra device memory at cfg2: %.1f MiB (fast %.1f MiB)" % (extra, used[0] / 2 ** 20))
    assert extra < 250, extra


def test_driver_worker_end_to_end(fold1, tmp_path):
    """The testbprmf-structured driver: text folds -> loadSparseR ->
    matBinarize -> device Sampler -> BPRMF.train -> scores (testbprmf.py:32-52)."""
    from collaborativefilteringusingtensorflow_amd.drivers import testbprmf
    for tag in ("train", "test"):
        ip, ix = fold1[tag + "_indptr"], fold1[tag + "_indices"]
        name = "ratings__1_%s.txt" % ("tra" if tag == "train" else "tst")
        with open(tmp_path / name, "w") as f:
            for u in range(943):
                for it in ix[ip[u]:ip[u + 1]]:
                    f.write("%d\t%d\t4.0\n" % (u, it))
            f.write("0\t0\t2.0\n")            # below the threshold: dropped by matBinarize
    old = testbprmf.n_factors
    testbprmf.n_factors = 32
    try:
        scores = testbprmf.worker(0, 943, 1682, str(tmp_path) + "/")
    finally:
        testbprmf.n_factors = old
    assert len(scores) == 5 and scores[4] > 0.2   # ndcg@10 after 50 epochs


def test_fold_parallel_driver_replicas(fold1, tmp_path):
    """run_folds(parallel=True): folds as independent spawned GPU replicas
    (CF_DEVICE = fold % devices) with the reference's ave@N / std@N report
    (testbprmf.py:113-125); two copies of fold 1 give identical-data replicas."""
    from collaborativefilteringusingtensorflow_amd.drivers import testbprmf
    from collaborativefilteringusingtensorflow_amd.drivers._common import run_folds
    for fold in (1, 2):
        for tag in ("train", "test"):
            ip, ix = fold1[tag + "_indptr"], fold1[tag + "_indices"]
            name = "ratings__%d_%s.txt" % (fold, "tra" if tag == "train" else "tst")
            with open(tmp_path / name, "w") as f:
                for u in range(943):
                    for it in ix[ip[u]:ip[u + 1]]:
                        f.write("%d\t%d\t4.0\n" % (u, it))
    aves, stds = run_folds(testbprmf.worker, 943, 1682, str(tmp_path) + "/", 2, 10,
                           testbprmf.eval_metrics, parallel=True)
    assert aves.shape == (5,) and aves[4] > 0.2
    # same data; the drivers' samplers are unseeded like the reference's
    # (SURVEY 0.10), so the two replicas differ only by sampling noise
    assert np.all(stds <= 0.03), stds


def test_fold_parallel_replicas_match_oracle(fold1, tmp_path):
    """Each spawned replica of run_folds(parallel=True) against the oracle:
    three folds (copies of ml-100k fold 1 written as text) train
    concurrently in spawned processes with the deterministic cfg1 worker
    (reference sampler stream for seed 11, seeded init); every replica's five
    ranking metrics must equal the oracle's committed cfg1 metrics
    (tests/golden/cfg1_oracle_metrics.json) within the north star's 0.2 %,
    and the replicas must agree with each other (testbprmf.py:113-125)."""
    from collaborativefilteringusingtensorflow_amd.drivers._common import run_folds
    from _replica_worker import cfg1_config, seeded_worker
    folds = 3
    for fold in range(1, folds + 1):
        for tag in ("train", "test"):
            ip, ix = fold1[tag + "_indptr"], fold1[tag + "_indices"]
            name = "ratings__%d_%s.txt" % (fold, "tra" if tag == "train" else "tst")
            with open(tmp_path / name, "w") as f:
                for u in range(943):
                    for it in ix[ip[u]:ip[u + 1]]:
                        f.write("%d\t%d\t4.0\n" % (u, it))
    g = cfg1_config()
    ref = np.array([g["metrics"][m] for m in g["config"]["metrics"]])
    import multiprocessing
    ctx = multiprocessing.get_context("spawn")
    # run_folds collects the replicas' score vectors through its queue; call
    # the entry the same way so the per-replica scores are visible here
    q = ctx.Queue()
    from collaborativefilteringusingtensorflow_amd.drivers._common import _fold_entry
    procs = [ctx.Process(target=_fold_entry, args=(seeded_worker, f, 0, 943, 1682,
                                                   str(tmp_path) + "/", q)) for f in range(folds)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(folds):
        f, sc, err = q.get(timeout=100)
        assert err is None, (f, err)
        got[f] = np.array(sc)
    for p in procs:
        p.join()
    for f in range(folds):
        rel = np.abs(got[f] - ref) / np.abs(ref)
        print("replica", f, got[f], "max rel vs oracle", rel.max())
        assert np.all(rel <= 2e-3), (f, got[f], ref)
        # same data and stream: the replicas differ only by the order of the
        # hot rows' float atomics (fast path), far inside the tolerance
        assert np.all(np.abs(got[f] - got[0]) <= 1e-3 * np.abs(ref)), (got[f], got[0])
    # and the driver's own ave@N / std@N path over the same replicas
    aves, stds = run_folds(seeded_worker, 943, 1682, str(tmp_path) + "/", folds, 10,
                           g["config"]["metrics"], parallel=True)
    assert np.all(np.abs(aves - ref) <= 2e-3 * np.abs(ref)), (aves, ref)
    assert np.all(stds <= 1e-3 * np.abs(ref)), stds


@pytest.mark.parametrize("name", ["prigp", "cplr"])
def test_tuple_models_train(fold1, name):
    """PRIGP / CPLR drop-ins (prigp.py:172-228, cplr_u.py:179-291): similarity
    preprocessing, their samplers, host-fed cf_step_plr; a few epochs on
    ml-100k fold 1 train well above random (random ndcg@10 ~ 0.01)."""
    tra, tst = matrices(fold1)
    if name == "prigp":
        from collaborativefilteringusingtensorflow_amd.prigp import PRIGP
        m = PRIGP(943, 1682, 5, 10, 'cv', ['pre', 'recall', 'map', 'mrr', 'ndcg'], 10., 0.1, 32,
                  1000, max_iter=8, seed=3, verbose=False)
    else:
        from collaborativefilteringusingtensorflow_amd.cplr import CPLR
        m = CPLR(943, 1682, 200, 10, 'cv', ['pre', 'recall', 'map', 'mrr', 'ndcg'], 1., 1., 1., 0.1,
                 32, 100, max_iter=3, seed=3, verbose=False)
    scores = m.train(1, tra, tst)
    m.close()
    print(name, scores)
    assert len(scores) == 5 and scores[4] > 0.1
