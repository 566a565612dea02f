"""Two ranks of the user-sharded data-parallel step on the REAL engine.

Both ranks share device 0 of the one-GPU test box and all-reduce the bound
item-gradient tensor with gloo (RCCL refuses two ranks on one device; on the
8-GPU node bench.py uses nccl = RCCL with the same ShardedStep).  After K
steps every rank's user shard and the replicated item table must equal the
float64 oracle run on the concatenated batches (1e-5 relative).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fold, batches, U0, V0, model, item_reduce, q, exchange="allreduce",
            backend="gloo", item_slots=0, opts=None, pieces=1):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from collaborativefilteringusingtensorflow_amd.distributed import (make_gpu_sharded,
                                                                       shard_users, local_csr)
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    if backend == "nccl":   # RCCL accepts a one-rank communicator on device 0
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                                world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                                world_size=world)
    ip, ix = fold["train_indptr"], fold["train_indices"]
    u0, u1 = shard_users(ip, world, rank)
    lip, lix = local_csr(ip, ix, u0, u1)
    W = batches[0][1].shape[1]
    kw = dict(reg=0.05) if model == "bpr" else dict(margin=1.0, reg_cov=1.0, clip_norm=1.0)
    e = Engine(model, u1 - u0, 1682, U0.shape[1], n_neg=W, dense_item_apply=True,
               seed=10 + rank, **kw)
    e.set_option("item_reduce", item_reduce)
    e.set_option("item_slots", item_slots)
    for k, v in (opts or {}).items():
        e.set_option(k, v)
    e.set_interactions(lip, lix)
    e.set_table("user", U0[u0:u1])
    e.set_table("item", V0)
    step, items = make_gpu_sharded(e, 1682, U0.shape[1], False, torch.device("cuda", 0),
                                   exchange=exchange, pieces=pieces)
    e.profile(True)
    for pairs, negs in batches:
        mine = (pairs[:, 0] >= u0) & (pairs[:, 0] < u1)
        lp = pairs[mine].copy()
        lp[:, 0] -= u0
        step(pairs=lp, negs=negs[mine])
    step.sync_state()     # rs_ag: the owners' accumulator rows to every rank
    torch.cuda.synchronize()
    e.profile(False)
    q.put((rank, u0, u1, e.get_table("user"), e.get_table("item"), e.get_table("acc_item"),
           e.profile_read("item_reduce")[1]))
    e.close()
    dist.barrier()
    dist.destroy_process_group()


def _oracle_run(model, batches, U0, V0):
    from oracle import cf_oracle as O
    U, V = U0.astype(np.float64), V0.astype(np.float64)
    AU, AV = np.full_like(U, 0.1), np.full_like(V, 0.1)
    for pairs, negs in batches:
        if model == "bpr":
            O.bpr_step(U, V, AU, AV, pairs, negs, 0.05)
        else:
            O.cml_step(U, V, AU, AV, pairs, negs, 1.0, 1.0, 1.0)
    return U, V, AU, AV


def _check_elementwise(got, ref, rtol=1e-5, atol=1e-6):
    """Elementwise |got - ref| <= atol + rtol |ref| against the float64 oracle
    (north star: 1e-5 relative on fp32 embeddings; atol covers elements that
    cancel to ~0 after updates of ~0.1).  CML trajectories get rtol 5e-5,
    atol 3e-6: the oracle itself run in float32 leaves the strict band
    (tests/test_oracle.py::test_fp32_oracle_drift_bounds_cml_tolerance)."""
    err = np.abs(got.astype(np.float64) - ref)
    bad = err > atol + rtol * np.abs(ref)
    assert not bad.any(), (int(bad.sum()), float(err.max()))


@pytest.mark.parametrize("item_slots", [0, 1, 2], ids=["rows", "records", "rows-pos-sort"])
@pytest.mark.parametrize("exchange", ["allreduce", "rs_ag"])
@pytest.mark.parametrize("model,stream", [("bpr", "rank_b100_w5"), ("cml", "rank_b50_w5")])
def test_one_rank_rccl_sharded_step(fold1, streams, model, stream, exchange, item_slots):
    """The RCCL path itself (nccl backend, world size 1 on device 0): the
    asynchronous collectives, the user apply beside them and the stream
    ordering of cf_step_local_apply / cf_step_items(_range) against them."""
    from oracle import cf_oracle as O
    rng = np.random.RandomState(9)
    d = 32
    U0 = O.init_table(rng, (943, d), truncated=(model != "cml"))
    V0 = O.init_table(rng, (1682, d), truncated=(model != "cml"))
    batches = [(streams[stream + "/pairs"][s], streams[stream + "/negs"][s]) for s in range(8)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    # rows-pos-sort: slot rows + positive-sorted gradients (the item reduce sums
    # the positive partials; CML forced onto the phased kernel where it applies)
    opts = {"pos_sort": 1, "grad_path": 2} if item_slots == 2 else {"pos_sort": 0}
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), fold1, batches, U0, V0, model, 1, q,
                                          exchange, "nccl", min(item_slots, 1) if item_slots < 2 else 0,
                                          opts))
    p.start()
    rank, u0, u1, Ul, Vr, AVr, _ = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    U, V, AU, AV = _oracle_run(model, batches, U0, V0)
    tol = dict(rtol=5e-5, atol=3e-6) if model == "cml" else {}
    _check_elementwise(Ul, U, **tol)
    _check_elementwise(Vr, V, **tol)
    _check_elementwise(AVr, AV, **tol)


@pytest.mark.parametrize("item_reduce,exchange,psort", [(1, "allreduce", 0), (2, "allreduce", 0),
                                                        (0, "allreduce", 0), (1, "rs_ag", 0),
                                                        (1, "allreduce", 1), (1, "rs_ag", 1)],
                         ids=["reduce", "store-singletons", "atomic", "reduce-scatter", "reduce-pos-sort",
                              "reduce-scatter-pos-sort"])
@pytest.mark.parametrize("model,stream", [("bpr", "rank_b100_w5"), ("cml", "rank_b50_w5")])
def test_two_rank_sharded_engine_equals_global_step(fold1, streams, model, stream, item_reduce,
                                                    exchange, psort):
    from oracle import cf_oracle as O
    rng = np.random.RandomState(8)
    d = 24
    U0 = O.init_table(rng, (943, d), truncated=(model != "cml"))
    V0 = O.init_table(rng, (1682, d), truncated=(model != "cml"))
    batches = [(streams[stream + "/pairs"][s], streams[stream + "/negs"][s]) for s in range(8)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    opts = {"pos_sort": 1, "grad_path": 2} if psort else {"pos_sort": 0}
    procs = [ctx.Process(target=_worker, args=(r, 2, port, fold1, batches, U0, V0, model, item_reduce, q,
                                               exchange, "gloo", 0, opts))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    U, V, AU, AV = _oracle_run(model, batches, U0, V0)
    for rank, u0, u1, Ul, Vr, AVr, _ in res:
        tol = dict(rtol=5e-5, atol=3e-6) if model == "cml" else {}
        _check_elementwise(Ul, U[u0:u1], **tol)
        _check_elementwise(Vr, V, **tol)
        _check_elementwise(AVr, AV, **tol)
    assert np.array_equal(res[0][4], res[1][4])   # replicas bit-identical


@pytest.mark.parametrize("pieces", [1, 3, 7])
def test_two_rank_item_reduce_in_pieces(fold1, streams, pieces):
    """Two ranks (gloo, one device) with the multi-rank item reduce in
    pieces: each piece's rows [item_r0, item_r1) reduced by its own launch
    and all-reduced across the ranks before the next piece, then the
    replicated item Adagrad.  Batches of six concatenated captured reference
    batches (600 pairs, W = 5), so each rank's ~300 pairs take pos_sort's
    dense item apply -- the path the pieces split.  Both ranks' shards and
    the replicated item table must equal the float64 oracle on the global
    batches, and the replicas each other bitwise (round-4 ADVICE: pieces were
    only ever checked at world 1)."""
    from oracle import cf_oracle as O
    rng = np.random.RandomState(12)
    d = 16
    U0 = O.init_table(rng, (943, d), truncated=True)
    V0 = O.init_table(rng, (1682, d), truncated=True)
    P, N = streams["rank_b100_w5/pairs"], streams["rank_b100_w5/negs"]
    batches = [(P[6 * s:6 * s + 6].reshape(-1, 2), N[6 * s:6 * s + 6].reshape(-1, 5)) for s in range(4)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    opts = {"pos_sort": 1, "grad_path": 2}
    procs = [ctx.Process(target=_worker, args=(r, 2, port, fold1, batches, U0, V0, "bpr", 1, q,
                                               "allreduce", "gloo", 0, opts, pieces))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    U, V, AU, AV = _oracle_run("bpr", batches, U0, V0)
    for rank, u0, u1, Ul, Vr, AVr, n_red in res:
        assert n_red == 4 * pieces, (rank, n_red)   # the pieces ran as separate launches
        _check_elementwise(Ul, U[u0:u1])
        _check_elementwise(Vr, V)
        _check_elementwise(AVr, AV)
    assert np.array_equal(res[0][4], res[1][4])


def _draw_ahead_worker(port, fold, q, exchange="allreduce", W=2, opts=None):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from collaborativefilteringusingtensorflow_amd.distributed import make_gpu_sharded
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    ip, ix = fold["train_indptr"], fold["train_indices"]
    out = []
    for ahead in (True, False):
        e = Engine("bpr", 943, 1682, 16, n_neg=W, reg=0.05, dense_item_apply=True, seed=77)
        for k, v in (opts or {}).items():
            e.set_option(k, v)
        e.set_interactions(ip, ix)
        e.init_params(0.0, 0.1, seed=5)
        step, _ = make_gpu_sharded(e, 1682, 16, False, torch.device("cuda", 0), exchange=exchange)
        step.draw_ahead = ahead
        for _ in range(9):
            step(batch_size=120)
        torch.cuda.synchronize()
        state = e.sampler_state()
        nxt = e.sample(120)           # drops a drawn-ahead batch, rewinds the sampler
        loss = e.take_loss()
        for _ in range(2):            # steps after the drop see clean counts
            step(batch_size=120)
        torch.cuda.synchronize()
        out.append((e.get_table("user"), e.get_table("item"), e.get_table("acc_user"), state,
                    nxt[0], nxt[1], loss))
        e.close()
    q.put(out)
    dist.destroy_process_group()


@pytest.mark.parametrize("exchange,W,psort", [("allreduce", 2, 0), ("rs_ag", 2, 0), ("allreduce", 5, 1),
                                             ("rs_ag", 1, 1)])
def test_draw_ahead_split_step_equals_plain_split_step(fold1, exchange, W, psort):
    """cf_step_local_grad / cf_step_local_apply(next_B) (all-reduce) or
    cf_step_local_draw (reduce-scatter): the batch drawn ahead is the one the
    sampler would draw next; dropping it rewinds."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    # psort: the drawn-ahead batch's positives are counted in cntP, and the
    # drop (cf_sample) must clear them too
    p = ctx.Process(target=_draw_ahead_worker, args=(_free_port(), fold1, q, exchange, W,
                                                     {"pos_sort": psort}))
    p.start()
    a, b = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    for x, y in zip(a[:3], b[:3]):   # float-atomic item sums: last-bit order effects only
        assert np.abs(x - y).max() <= 1e-6 * np.abs(y).max()
    assert a[3] == b[3]
    assert np.array_equal(a[4], b[4]) and np.array_equal(a[5], b[5])
    assert abs(a[6] - b[6]) <= 1e-6 * abs(b[6])


def _pieces_worker(port, fold, q, pieces_list, one_call=False):
    """Host-fed steps (batches from the engine's own device sampler,
    cf_sample) through the sharded step with the item reduce in P pieces,
    each step checked against one float64 oracle step from the engine's own
    fp32 tables within the a-priori fp32 bound E (LocalStepCheck).  one_call:
    the one-call cf_step_local (no caller collective between pieces) +
    cf_step_items instead of ShardedStep."""
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from collaborativefilteringusingtensorflow_amd.distributed import make_gpu_sharded
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    from tests.conftest import LocalStepCheck
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    ip, ix = fold["train_indptr"], fold["train_indices"]
    out = []
    for P in pieces_list:
        e = Engine("bpr", 943, 1682, 32, n_neg=1, reg=0.05, dense_item_apply=True, seed=91)
        e.set_option("pos_sort", 1)
        e.set_interactions(ip, ix)
        e.init_params(0.0, 0.1, seed=6)
        step, _ = make_gpu_sharded(e, 1682, 32, False, torch.device("cuda", 0), pieces=P)
        if one_call:
            e.set_option("item_pieces", P)
        chk = LocalStepCheck(reg=0.05)
        e.profile_reset()
        e.profile(True)
        for s in range(6):
            pairs, negs, _ = e.sample(2048)
            chk.before(e)
            if one_call:
                e.step_local(pairs=pairs, negs=negs)
                e.step_items()
            else:
                step(pairs=pairs, negs=negs)
            torch.cuda.synchronize()
            chk.after(e, pairs, negs, e.take_loss(), "P=%d step %d" % (P, s))
        e.profile(False)
        out.append((P, e.profile_read("item_reduce")[1], chk.worst))
        e.close()
    q.put(out)
    dist.destroy_process_group()


@pytest.mark.parametrize("one_call", [False, True], ids=["sharded-step", "one-call-step-local"])
def test_one_rank_rccl_item_reduce_in_pieces(fold1, one_call):
    """The item reduce in pieces of item rows (cf_step_item_reduce,
    AllReduceItems(pieces=P)), each piece's all-reduce issued on RCCL right
    after it (one rank on device 0, pos_sort's dense item apply, hot items
    past capP).  Every step of every P is checked against the float64 oracle
    within the a-priori fp32 bound E, not against another fast-path run: a
    piece boundary that dropped or doubled a row's contribution lands outside
    E (tests/test_fp32_bound.py), untouched rows must be bit-identical.
    one-call: cf_step_local with item_pieces > 1 reduces the deferred pieces
    itself (round-4 ADVICE: it used to leave the engine in the split state).
    The r04j red run that made the old bitwise self-comparison non-bitwise is
    profiles/r04/red_runs/r04j_pytest.log."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_pieces_worker, args=(_free_port(), fold1, q, (1, 3, 7), one_call))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    for P, n_red, worst in res:
        # P = 1: one whole reduce per step; P > 1: deferred, P piece launches
        assert n_red == 6 * P, (P, n_red)
        assert worst <= 1.0, (P, worst)


def _apr_worker(rank, world, port, fold, batches, U0, V0, q, backend, exchange="allreduce", opts=None):
    """AMF apr across ranks: each rank's users, the item rows' Δ from the
    global batch (cf_step_local_apr_embed + the all-reduce of the bound
    buffer inside ShardedStep)."""
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from collaborativefilteringusingtensorflow_amd.distributed import (make_gpu_sharded,
                                                                       shard_users, local_csr)
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                                world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                                world_size=world)
    ip, ix = fold["train_indptr"], fold["train_indices"]
    u0, u1 = shard_users(ip, world, rank)
    lip, lix = local_csr(ip, ix, u0, u1)
    W = batches[0][1].shape[1]
    e = Engine("amf", u1 - u0, 1682, U0.shape[1], n_neg=W, dense_item_apply=True, seed=10 + rank,
               reg=0.05, reg_adv=1.0, epsilon=0.5, amf_mode="apr")
    for k, v in (opts or {}).items():
        e.set_option(k, v)
    e.set_interactions(lip, lix)
    e.begin_phase(1)
    e.set_table("user", U0[u0:u1])
    e.set_table("item", V0)
    step, items = make_gpu_sharded(e, 1682, U0.shape[1], False, torch.device("cuda", 0), exchange=exchange)
    for pairs, negs in batches:
        mine = (pairs[:, 0] >= u0) & (pairs[:, 0] < u1)
        lp = pairs[mine].copy()
        lp[:, 0] -= u0
        step(pairs=lp, negs=negs[mine])
    step.sync_state()
    torch.cuda.synchronize()
    q.put((rank, u0, u1, e.get_table("user"), e.get_table("item"), e.get_table("acc_item")))
    e.close()
    dist.barrier()
    dist.destroy_process_group()


def _apr_oracle(batches, U0, V0):
    from oracle import cf_oracle as O
    U, V = U0.astype(np.float64), V0.astype(np.float64)
    AU, AV = np.full_like(U, 0.1), np.full_like(V, 0.1)
    for pairs, negs in batches:
        O.amf_apr_step(U, V, AU, AV, pairs, negs, 0.05, 0.5, reg_adv=1.0)
    return U, V, AU, AV


def _apr_tables(seed, d=24):
    from oracle import cf_oracle as O
    rng = np.random.RandomState(seed)
    return O.init_table(rng, (943, d)), O.init_table(rng, (1682, d))


@pytest.mark.parametrize("item_reduce", [1, 0], ids=["reduce", "atomic"])
def test_one_rank_rccl_apr(fold1, streams, item_reduce):
    """AMF apr on the multi-rank code path over RCCL (world 1): the embed
    pass, the all-reduce of the bound buffer, the gradient launch reading
    every item row's Δ from it, the buffer cleared for the next step."""
    U0, V0 = _apr_tables(21)
    batches = [(streams["rank_b100_w5/pairs"][s], streams["rank_b100_w5/negs"][s]) for s in range(8)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_apr_worker, args=(0, 1, _free_port(), fold1, batches, U0, V0, q, "nccl",
                                              "allreduce", {"item_reduce": item_reduce}))
    p.start()
    rank, u0, u1, Ul, Vr, AVr = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    U, V, AU, AV = _apr_oracle(batches, U0, V0)
    _check_elementwise(Ul, U)
    _check_elementwise(Vr, V)
    _check_elementwise(AVr, AV)


@pytest.mark.parametrize("exchange", ["allreduce", "rs_ag"])
def test_two_rank_apr_equals_global_step(fold1, streams, exchange):
    """Two ranks (gloo, one device): a row seen once on each rank is a
    duplicate of the global batch, so its Δ must come from the summed
    buffer -- every rank's tables equal the oracle's apr steps on the
    concatenated batches."""
    U0, V0 = _apr_tables(22)
    batches = [(streams["rank_b100_w5/pairs"][s], streams["rank_b100_w5/negs"][s]) for s in range(8)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_apr_worker, args=(r, 2, port, fold1, batches, U0, V0, q, "gloo", exchange))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    U, V, AU, AV = _apr_oracle(batches, U0, V0)
    for rank, u0, u1, Ul, Vr, AVr in res:
        _check_elementwise(Ul, U[u0:u1])
        _check_elementwise(Vr, V)
        _check_elementwise(AVr, AV)
    assert np.array_equal(res[0][4], res[1][4])
