"""GPU parity of the positive-sorted gradient (cf_set_option "pos_sort").

The draw counts each pair's positive item apart from the negatives, psort
orders the pairs by positive item, and the gradient launch sums the pairs of
one block that share a positive item in LDS: one partial row per (block,
item) instead of one slot row (or float atomics) per occurrence.  The step is
still TF1's dedup-sum + SparseApplyAdagrad (bprmf.py:74-88), so every case is
checked against the float64 oracle: each BPR / AMF step from the engine's own
pre-step tables within the a-priori fp32 bound of oracle/fp32_bound.py
(conftest.LocalStepCheck), and the trajectory at the north star's 1e-5,
elementwise (|gpu - oracle| <= 1e-6 + 1e-5 |oracle| on every element of every
table; the per-step loss within 1e-5) on the reference's captured batches,
plus hot items whose partials overflow their slot range (their trajectory
band adds the same a-priori bound carried over the steps), items seen only
as positives, and the device-sampled pipeline (draw fused into the apply
launch).
"""
import numpy as np
import pytest

from conftest import CML_TRAJ, LocalStepCheck, assert_close, get_stream
from oracle import cf_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def make(model, fold1, d, W, opts, **kw):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    e = Engine(model, int(fold1["n_users"]), int(fold1["n_items"]), d, n_neg=W, seed=7, **kw)
    e.set_option("item_slots", 0)
    for k, v in opts.items():
        e.set_option(k, v)
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    return e


def tables(fold1, d, seed, truncated=True):
    rng = np.random.RandomState(seed)
    U = O.init_table(rng, (int(fold1["n_users"]), d), truncated=truncated)
    V = O.init_table(rng, (int(fold1["n_items"]), d), truncated=truncated)
    return U, V


def psort_launches(e):
    return e.profile_read("psort")[1]


def run_steps(model, fold1, batches, d, opts, amf_switch=None, forward_bound=False, **kw):
    """Engine steps on host-fed batches.  BPR / AMF: every step against the
    float64 oracle from the engine's own pre-step tables within the a-priori
    fp32 bound (conftest.LocalStepCheck); the whole trajectory against the
    float64 oracle in the strict band -- plus, with ``forward_bound``, the
    same a-priori bound carried over the steps (oracle/fp32_bound.py): a
    Zipf-head row's fp32 rounding, amplified over steps, leaves the strict
    band in every summation order, the float32 oracle's own included."""
    from oracle import fp32_bound as FB
    W = batches[0][1].shape[1]
    U, V = tables(fold1, d, 3, truncated=(model != "cml"))
    e = make(model, fold1, d, W, opts, **kw)
    e.set_table("user", U)
    e.set_table("item", V)
    e.profile_reset()
    e.profile(True)
    U64, V64 = U.astype(np.float64), V.astype(np.float64)
    AU, AV = np.full_like(U64, 0.1), np.full_like(V64, 0.1)
    E = FB.zero_bounds(U64, V64) if forward_bound else None
    if model in ("bpr", "amf"):
        local = LocalStepCheck(kw["reg"], adversarial=None if model == "bpr" else False,
                               reg_adv=kw.get("reg_adv", 1.0))
    else:
        local = LocalStepCheck(model="cml", margin=kw["margin"], reg_cov=kw["reg_cov"],
                               clip_norm=kw["clip_norm"], use_rank_weight=kw["use_rank_weight"])
    adv = False
    for s, (pairs, negs) in enumerate(batches):
        if amf_switch is not None and s == amf_switch:
            e.begin_phase(1)
            adv = True
            AU[...] = 0.1
            AV[...] = 0.1
            local.T, local.adversarial = None, True
        local.before(e)
        lg = e.step(pairs, negs)
        local.after(e, pairs, negs, lg, "step %d" % s)
        if model == "bpr":
            if E is not None:
                lo = FB.bpr_step_bounded(U64, V64, AU, AV, E, pairs, negs, kw["reg"])
            else:
                lo = O.bpr_step(U64, V64, AU, AV, pairs, negs, kw["reg"])
        elif model == "amf":
            lo = O.amf_step(U64, V64, AU, AV, pairs, negs, kw["reg"], adv, reg_adv=kw.get("reg_adv", 1.0))
        else:
            lo = O.cml_step(U64, V64, AU, AV, pairs, negs, kw["margin"], kw["reg_cov"], kw["clip_norm"],
                            use_rank_weight=kw["use_rank_weight"])
        assert abs(lg - lo) <= RTOL * abs(lo) + 1e-6, (s, lg, lo)
    e.profile(False)
    n_ps = psort_launches(e)
    tol = CML_TRAJ if model == "cml" else {}
    for t, o in (("user", U64), ("item", V64), ("acc_user", AU), ("acc_item", AV)):
        assert_close(e.get_table(t), o, t, bound=None if E is None else E[t], **tol)
    e.close()
    return n_ps


def stream_batches(streams, name, K):
    st = get_stream(streams, name)
    return [(st["pairs"][s], st["negs"][s]) for s in range(K)]


@pytest.mark.parametrize("cap", [1, 8])
@pytest.mark.parametrize("name,d,reg", [("rank_b100_w1", 32, 0.1), ("rank_b100_w5", 64, 0.05),
                                        ("uij_b100", 16, 0.02)])
def test_bpr_pos_sort_matches_oracle(fold1, streams, name, d, reg, cap):
    n = run_steps("bpr", fold1, stream_batches(streams, name, 40), d,
                  {"pos_sort": 1, "slot_max_pos": cap}, reg=reg)
    assert n == 40   # the sorted kernel ran every step


def test_amf_pos_sort_across_phase_switch(fold1, streams):
    n = run_steps("amf", fold1, stream_batches(streams, "rank_b100_w5", 40), 128,
                  {"pos_sort": 1}, amf_switch=20, reg=0.05, reg_adv=1.0)
    assert n == 40


def test_cml_pos_sort_phased(fold1, streams):
    """CML at W=5 on the phased kernel (grad_path 2; auto keeps the generic
    one, where pos_sort does not apply) with the clip in every update."""
    n = run_steps("cml", fold1, stream_batches(streams, "rank_b50_w5", 40), 50,
                  {"pos_sort": 1, "grad_path": 2}, margin=1.0, reg_cov=1.0, clip_norm=1.0,
                  use_rank_weight=True)
    assert n == 40


def test_pos_sort_inactive_paths_unchanged(fold1, streams):
    """Where pos_sort does not apply (generic kernel, CML auto at W=5) the
    option is ignored and the step is the plain one."""
    n = run_steps("bpr", fold1, stream_batches(streams, "rank_b100_w1", 10), 32,
                  {"pos_sort": 1, "grad_path": 1}, reg=0.1)
    assert n == 0
    n = run_steps("cml", fold1, stream_batches(streams, "rank_b50_w5", 10), 50,
                  {"pos_sort": 1}, margin=1.0, reg_cov=1.0, clip_norm=1.0, use_rank_weight=True)
    assert n == 0


def hot_batch(fold1, rng, n_pos, n_neg_hot, hot=49, B=900):
    """Item `hot` as the positive of the first n_pos pairs (users who rated
    it) and the negative of n_neg_hot more; other pairs ordinary."""
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    raters = [u for u in range(943) if hot in set(ix[ip[u]:ip[u + 1]].tolist())]
    pairs, negs = [], []
    for r in range(B):
        if r < n_pos:
            u = raters[rng.randint(len(raters))]
            row = set(ix[ip[u]:ip[u + 1]].tolist())
            pairs.append([u, hot])
        else:
            u = int(rng.randint(943))
            while ip[u + 1] == ip[u] or hot in set(ix[ip[u]:ip[u + 1]].tolist()):
                u = int(rng.randint(943))
            row = set(ix[ip[u]:ip[u + 1]].tolist())
            pairs.append([u, int(ix[ip[u] + rng.randint(ip[u + 1] - ip[u])])])
        if n_pos <= r < n_pos + n_neg_hot:
            negs.append([hot])
        else:
            negs.append([next(int(x) for x in rng.randint(0, 1682, 64) if x not in row and x != hot)])
    return np.array(pairs, np.int32), np.array(negs, np.int32)


@pytest.mark.parametrize("cap,slot_max", [(1, 3), (8, 32), (64, 32)])
@pytest.mark.parametrize("n_pos,n_neg_hot", [(600, 300), (600, 0), (5, 0)])
def test_pos_sort_hot_item(fold1, cap, slot_max, n_pos, n_neg_hot):
    """A hot positive spanning ~38 gradient blocks: partials 0..cap-1 in
    slots, the rest float atomics; with n_neg_hot 0 the item is no pair's
    negative, so its rank-0 positive owns the apply."""
    rng = np.random.RandomState(n_pos + n_neg_hot + cap)
    batches = [hot_batch(fold1, rng, n_pos, n_neg_hot) for _ in range(3)]
    n = run_steps("bpr", fold1, batches, 16, {"pos_sort": 1, "slot_max_pos": cap, "slot_max": slot_max},
                  forward_bound=True, reg=0.02)
    assert n == 3


def test_pos_sort_device_pipeline_equals_plain(fold1):
    """cf_train_steps (device draw fused into the apply launch, the psort
    launches between) trains the same model as the plain path from the same
    state and sampler seed: same batches, sums equal up to fp32 order."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    out = []
    for ps in (0, 1):
        e = Engine("bpr", 943, 1682, 64, n_neg=1, reg=0.05, seed=21)
        e.set_option("item_slots", 0)
        e.set_option("pos_sort", ps)
        e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
        e.init_params(0.0, 0.1, truncated=True, seed=1)
        e.profile_reset()
        e.profile(True)
        loss = e.train_steps(2048, 30)
        e.profile(False)
        out.append((loss, e.get_table("user"), e.get_table("item"), e.get_table("acc_item"),
                    psort_launches(e)))
        e.close()
    (l0, U0, V0, A0, n0), (l1, U1, V1, A1, n1) = out
    assert n0 == 0 and n1 == 30
    assert abs(l1 - l0) <= 1e-5 * abs(l0)
    for name, a, b in (("user", U1, U0), ("item", V1, V0), ("acc_item", A1, A0)):
        assert_close(a, b, name)


def test_pos_sort_device_pipeline_matches_oracle(fold1):
    """The same path against the oracle replaying the engine's own draws."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    d, reg, B = 32, 0.05, 1024
    e = Engine("bpr", 943, 1682, d, n_neg=1, reg=reg, seed=33)
    e.set_option("pos_sort", 1)
    e.set_option("item_slots", 0)
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    U, V = tables(fold1, d, 5)
    e.set_table("user", U)
    e.set_table("item", V)
    # the sampler stream: draw K batches, rewind, train the same K on the device
    st = e.sampler_state()
    batches = [e.sample(B)[:2] for _ in range(12)]
    e.set_sampler_state(*st)
    e.train_steps(B, 12)
    U64, V64 = U.astype(np.float64), V.astype(np.float64)
    AU, AV = np.full_like(U64, 0.1), np.full_like(V64, 0.1)
    for pairs, negs in batches:
        O.bpr_step(U64, V64, AU, AV, pairs, negs, reg)
    for t, o in (("user", U64), ("item", V64), ("acc_user", AU), ("acc_item", AV)):
        assert_close(e.get_table(t), o, t)
    e.close()


def test_pos_sort_auto_by_batch_size():
    """Default (auto): on from 2^18 pairs per step, off below.  At 2^18 pairs
    on a 60K x 8K Zipf(0.8) graph the auto path (psort + partial rows, hot
    items past capP on float atomics) is checked against the float64 oracle
    replaying the engine's own draws -- the test through which the round-2
    owner race (a duplicated item applied twice) surfaced:

    * K single device-drawn steps, each from the engine's own pre-step tables
      within the one-step a-priori fp32 bound (conftest.LocalStepCheck: every
      element of every table, none excluded);
    * one two-step cf_train_steps call (the apply launch of step 1 draws and
      counts step 2) within the bound carried over its two steps, which stays
      finite on all but a handful of elements (asserted: <= 1 %; over three
      or more steps the carried accumulator bound outgrows the accumulators of
      the Zipf head and reads inf)."""
    from collaborativefilteringusingtensorflow_amd.engine import Engine, synth_graph
    from oracle import fp32_bound as FB
    nu, ni, d, reg = 60_000, 8_000, 64, 0.02
    ip, ix = synth_graph(nu, ni, 30.0, 0.8, 7, n_threads=8)
    e = Engine("bpr", nu, ni, d, n_neg=1, reg=reg, seed=3)
    e.set_interactions(ip, ix)
    e.init_params(0.0, 0.1, truncated=True, seed=1)
    e.profile_reset()
    e.profile(True)
    e.train_steps(1 << 16, 2)          # below the auto threshold
    n_small = psort_launches(e)
    B, K = 1 << 18, 3
    # one step at B first: the sampler moves to a new epoch when the batch
    # size changes, and (epoch, batch) alone does not restore that
    e.train_steps(B, 1)
    n_small += 1
    chk = LocalStepCheck(reg)
    for s in range(K):
        st = e.sampler_state()
        pairs, negs, _ = e.sample(B)     # the batch the next step draws
        e.set_sampler_state(*st)
        chk.before(e)
        loss = e.train_steps(B, 1)
        chk.after(e, pairs, negs, loss, "step %d" % s)
        if s == 0:   # the batches really overflow capP (8 partials) on their hottest positives
            cnt = np.bincount(pairs[:, 1], minlength=ni)
            off = np.cumsum(cnt) - cnt
            nparts = np.where(cnt > 0, (off + cnt - 1) // 16 - off // 16 + 1, 0)
            assert nparts.max() > 8, nparts.max()
    assert chk.excluded == 0
    # two pipelined steps in one call
    T = {t: e.get_table(t).astype(np.float64) for t in ("user", "item", "acc_user", "acc_item")}
    st = e.sampler_state()
    batches = [e.sample(B)[:2] for _ in range(2)]
    e.set_sampler_state(*st)
    loss = e.train_steps(B, 2)
    e.profile(False)
    n_big = psort_launches(e) - n_small
    assert n_small == 1 and n_big == K + 2
    E = FB.zero_bounds(T["user"], T["item"], acc_exact=True)
    lo = 0.0
    for pairs, negs in batches:
        lo += FB.bpr_step_bounded(T["user"], T["item"], T["acc_user"], T["acc_item"], E, pairs, negs, reg)
    assert abs(loss - lo) <= RTOL * abs(lo), (loss, lo)
    for t in T:
        assert_close(e.get_table(t), T[t], t, bound=E[t], max_excluded=0.01)
    e.close()


SPEC_MODELS = {"bpr": dict(reg=0.05), "amf": dict(reg=0.05, reg_adv=1.0),
               "cml": dict(margin=1.0, reg_cov=1.0, clip_norm=1.0)}


def _spec_engine(fold1, model, W, spec, det):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    e = Engine(model, 943, 1682, 32, n_neg=W, seed=41, **SPEC_MODELS[model])
    e.set_option("item_slots", 0)
    e.set_option("pos_sort", 1)
    e.set_option("spec_neg", spec)
    e.set_option("deterministic", det)
    e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
    e.init_params(0.0, 0.1, truncated=(model != "cml"), seed=2)
    return e


@pytest.mark.parametrize("model,W", [("bpr", 1), ("bpr", 5), ("amf", 1), ("amf", 5), ("cml", 1)])
def test_spec_neg_steps_match_oracle(fold1, model, W):
    """Speculative negative counts (cf_set_option "spec_neg", StepArgs::spec_ph):
    on ml-100k a heavy user's row holds up to ~40 % of the 1,682 items, so many
    first candidates are rejected and leave phantom occurrences (zeroed slot
    rows, phantom-only items' counts reset).  Each device-drawn step with
    phantoms is checked against one float64 oracle step on the same batch
    from the engine's own tables, within the a-priori fp32 bound
    (conftest.LocalStepCheck) -- BPR, AMF across its switch to the
    adversarial phase, and CML, whose apply clips every row it updates (an
    item touched only by phantoms must get no update and no clip)."""
    e = _spec_engine(fold1, model, W, 1, 0)
    kw = SPEC_MODELS[model]
    if model == "cml":
        chk = LocalStepCheck(model="cml", use_rank_weight=True, **kw)
    else:
        chk = LocalStepCheck(kw["reg"], adversarial=None if model == "bpr" else False,
                             reg_adv=kw.get("reg_adv", 1.0))
    e.profile(True)
    for s in range(10):
        if model == "amf" and s == 5:
            e.begin_phase(1)
            chk.T, chk.adversarial = None, True
        st = e.sampler_state()
        pairs, negs, _ = e.sample(2048)     # the batch the next step draws
        e.set_sampler_state(*st)
        chk.before(e)
        loss = e.train_steps(2048, 1)       # drawn on the device, with phantoms
        chk.after(e, pairs, negs, loss, "step %d" % s)
    e.profile(False)
    assert e.profile_read("psort")[1] == 10
    e.close()


def test_cml_spec_neg_on_and_off_each_match_oracle(fold1):
    """CML with speculative negative counts on and off (round 5 dropped CML
    from test_spec_neg_equals_plain_draw after its fast-path case put 6 user
    elements at 4.4x the CML trajectory band, profiles/r05/r05a/pytest.log;
    DESIGN 4.1).  Two fp32 runs whose duplicate sums add in different orders
    drift apart through CML's branch points (hinge, argmin, the rank weight's
    indicators), so a band between the two runs is not a sound check.  What
    must hold is that both settings draw the same batches and that every step
    of each is the float64 oracle's step from that engine's own tables within
    the a-priori bound (conftest.LocalStepCheck, ambiguous pairs excluded and
    counted) -- a phantom occurrence that leaked into a count, a slot row or a
    clip would land outside it."""
    kw = SPEC_MODELS["cml"]
    drawn = []
    for spec in (0, 1):
        e = _spec_engine(fold1, "cml", 1, spec, 0)
        chk = LocalStepCheck(model="cml", use_rank_weight=True, **kw)
        got = []
        for s in range(12):
            st = e.sampler_state()
            pairs, negs, _ = e.sample(2048)
            e.set_sampler_state(*st)
            chk.before(e)
            loss = e.train_steps(2048, 1)
            chk.after(e, pairs, negs, loss, "spec %d step %d" % (spec, s))
            got.append((pairs, negs))
        drawn.append(got)
        e.close()
    for s, ((p0, n0), (p1, n1)) in enumerate(zip(*drawn)):
        assert np.array_equal(p0, p1) and np.array_equal(n0, n1), s


@pytest.mark.parametrize("det", [0, 1], ids=["fast", "det"])
@pytest.mark.parametrize("model,W", [("bpr", 1), ("bpr", 5), ("amf", 1), ("amf", 5)])
def test_spec_neg_equals_plain_draw(fold1, model, W, det):
    """The same training with spec_neg on and off -- the draw is the same
    stream -- also across a discarded drawn-ahead batch (the batch size
    changes mid-run) and AMF's phase switch.  Fast path: equal up to fp32
    summation order.  Deterministic mode: bitwise equal -- it keeps the
    speculative counts off (a phantom would move an item whose only real
    occurrence shares its count onto the fixed-point summed path, changing
    its last bits; the deterministic result must not depend on a
    performance option)."""
    out = []
    for spec in (0, 1):
        e = _spec_engine(fold1, model, W, spec, det)
        e.profile(True)
        loss = e.train_steps(2048, 12)
        if model == "amf":
            e.begin_phase(1)                # the adversarial phase (amf.py:216-244)
        loss += e.train_steps(1024, 6)     # the pending 2048-pair draw is discarded
        loss += e.train_steps(2048, 6)
        e.profile(False)
        assert e.profile_read("psort")[1] == 24
        flags = e.step_path(2048)[1]
        assert flags["pos_sort"] and flags["deterministic"] == bool(det)
        out.append((loss, {t: e.get_table(t) for t in ("user", "item", "acc_user", "acc_item")}))
        e.close()
    (l0, T0), (l1, T1) = out
    if det:
        assert l1 == l0
        for t in T0:
            assert np.array_equal(T1[t], T0[t]), t
        return
    assert abs(l1 - l0) <= 1e-5 * abs(l0)
    for t in T0:
        assert_close(T1[t], T0[t], t)
