"""Two ranks of the user-sharded GBPR step with the cross-shard group exchange
on the REAL engine (cf_set_shard / cf_set_group_source / cf_xchg_*).

Both ranks share device 0 of the one-GPU test box and exchange through gloo
(host-staged all-to-alls; on an 8-GPU node the same GroupExchangeStep runs on
RCCL).  Host-fed: after K steps on the reference's captured GBPR batches
(sampler_gbpr.py, global group members) every rank's user shard, the item
table and the item bias must equal the float64 oracle on the concatenated
batches (1e-5 relative).  Device-sampled: the group members drawn on device
come from the item's users over both shards and the replicas stay identical.
"""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import assert_close
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fold, batches, U0, V0, b0, q, sampled, exchange="allreduce",
            pipelined=True, split=True, grad_path=0, backend="gloo"):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from collaborativefilteringusingtensorflow_amd.distributed import (make_gpu_group_exchange,
                                                                       shard_users, local_csr)
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    if backend == "nccl":   # RCCL accepts a one-rank communicator on device 0
        torch.cuda.set_device(0)
    dist.init_process_group(backend, init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=world)
    ip, ix = fold["train_indptr"], fold["train_indices"]
    bounds = [shard_users(ip, world, r)[0] for r in range(world)] + [943]
    u0, u1 = bounds[rank], bounds[rank + 1]
    lip, lix = local_csr(ip, ix, u0, u1)
    W, G = batches[0][1].shape[1], batches[0][2].shape[1]
    d = U0.shape[1]
    e = Engine("gbpr", u1 - u0, 1682, d, n_neg=W, gsize=G, rho=0.4, reg=0.01,
               dense_item_apply=True, seed=20 + rank)
    e.set_option("grad_path", grad_path)
    e.set_interactions(lip, lix)
    e.set_table("user", U0[u0:u1])
    e.set_table("item", V0)
    e.set_table("bias", b0)
    step, _items = make_gpu_group_exchange(e, world, rank, bounds, ip, ix, 1682, d, 100,
                                           torch.device("cuda", 0), exchange=exchange)
    step.pipelined = step.pipelined and pipelined
    step.split = split
    drawn = []
    if sampled == "steps":           # device-sampled steps only (pipelined count exchange)
        for _ in range(7):
            step(batch_size=64)
    elif sampled == "sizes":         # ... with the batch size changing between steps
        for bs in SIZES:
            step(batch_size=bs)
    elif sampled:
        for _ in range(6):
            pairs, negs, groups = e.sample(64)
            pairs = pairs.copy()
            pairs[:, 0] += u0          # sample() returns this rank's local user ids
            drawn.append((pairs, groups))
            step(batch_size=64)
    else:
        for pairs, negs, groups in batches:
            mine = (pairs[:, 0] >= u0) & (pairs[:, 0] < u1)
            lp = pairs[mine].copy()
            lp[:, 0] -= u0
            step(pairs=lp, negs=negs[mine], groups=groups[mine])
    step.sync_state()
    torch.cuda.synchronize()
    q.put((rank, u0, u1, e.get_table("user"), e.get_table("item"), e.get_table("bias"),
           e.get_table("acc_user"), drawn, e.get_table("acc_item"), e.get_table("acc_bias"), e.take_loss()))
    e.close()
    dist.barrier()
    dist.destroy_process_group()


SIZES = (64, 64, 48, 48, 64, 32, 32, 64)


def _run(fold1, batches, U0, V0, b0, sampled=False, exchange="allreduce", pipelined=True, split=True,
         grad_path=0, world=2, backend="gloo"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fold1, batches, U0, V0, b0, q, sampled, exchange,
                                               pipelined, split, grad_path, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("split", [True, False], ids=["split", "serial"])
@pytest.mark.parametrize("exchange", ["allreduce", "rs_ag"])
@pytest.mark.parametrize("stream", ["gbpr_b100_g1_w5", "gbpr_b100_g3_w2"])
def test_two_rank_group_exchange_equals_global_step(fold1, streams, stream, exchange, split):
    """split: the split exchange step (cf_xchg_grad_part 1 / 2, cf_xchg_finish_items);
    serial: cf_xchg_grad + cf_xchg_finish.  The ranks' losses sum to the
    global step's (each part writes its own half of the loss partials)."""
    _two_rank_global_step(fold1, streams, stream, exchange, split, 16, 0)


@pytest.mark.parametrize("split", [True, False], ids=["split", "serial"])
def test_two_rank_group_exchange_lds_kernel(fold1, streams, split):
    """The same at d = 64 on the LDS-staged GBPR kernel (grad_path 3), whose
    member pass filter serves the split step."""
    _two_rank_global_step(fold1, streams, "gbpr_b100_g1_w5", "allreduce", split, 64, 3)


@pytest.mark.parametrize("exchange", ["allreduce", "rs_ag"])
def test_one_rank_rccl_forced_split_step(fold1, streams, exchange):
    """The split exchange step on RCCL (nccl backend, one rank on device 0,
    split forced): its collectives are asynchronous there -- the member-row
    all-to-all runs beside gradient part 1, the item reduce beside the
    member-gradient all-to-all and the user finish -- so this checks their
    stream ordering against the float64 oracle (gloo, used by every multi-rank
    test, runs them synchronously)."""
    _two_rank_global_step(fold1, streams, "gbpr_b100_g1_w5", exchange, "force", 16, 0, world=1, backend="nccl")


def _two_rank_global_step(fold1, streams, stream, exchange, split, d, grad_path, world=2, backend="gloo"):
    from oracle import cf_oracle as O
    rng = np.random.RandomState(12)
    U0 = O.init_table(rng, (943, d))
    V0 = O.init_table(rng, (1682, d))
    b0 = O.init_table(rng, (1682,))
    batches = [(streams[stream + "/pairs"][s], streams[stream + "/negs"][s],
                streams[stream + "/groups"][s]) for s in range(8)]
    res = _run(fold1, batches, U0, V0, b0, exchange=exchange, split=split, grad_path=grad_path, world=world,
               backend=backend)
    U, V, b = U0.astype(np.float64), V0.astype(np.float64), b0.astype(np.float64)
    AU, AV, Ab = np.full_like(U, 0.1), np.full_like(V, 0.1), np.full_like(b, 0.1)
    lo = 0.0
    for pairs, negs, groups in batches:
        lo += O.gbpr_step(U, V, b, AU, AV, Ab, pairs, negs, groups, 0.4, 0.01)
    lg = sum(r[10] for r in res)
    assert abs(lg - lo) <= 1e-5 * abs(lo), (lg, lo)
    for rank, u0, u1, Ul, Vr, br, AUl, _, AVr, Abr, _ in res:
        assert_close(Ul, U[u0:u1], ("user", rank))
        assert_close(AUl, AU[u0:u1], ("acc_user", rank))
        assert_close(Vr, V, ("item", rank))
        assert_close(br, b, ("bias", rank))
        assert_close(AVr, AV, ("acc_item", rank))
        assert_close(Abr, Ab, ("acc_bias", rank))
    if world > 1:
        assert np.array_equal(res[0][4], res[1][4]) and np.array_equal(res[0][5], res[1][5])


def test_two_rank_device_sampled_groups_span_shards(fold1):
    from oracle import cf_oracle as O
    rng = np.random.RandomState(13)
    d = 16
    U0 = O.init_table(rng, (943, d))
    V0 = O.init_table(rng, (1682, d))
    b0 = O.init_table(rng, (1682,))
    dummy = [(np.zeros((1, 2), np.int32), np.zeros((1, 5), np.int32), np.zeros((1, 1), np.int32))]
    res = _run(fold1, dummy, U0, V0, b0, sampled=True)
    ip, ix = fold1["train_indptr"], fold1["train_indices"]
    cross = 0
    for rank, u0, u1, Ul, Vr, br, AUl, drawn, _, _, _ in res:
        assert np.all(np.isfinite(Ul)) and np.all(np.isfinite(Vr))
        for pairs, groups in drawn:
            for (u, i), g in zip(pairs, groups):
                assert u0 <= u < u1
                for gg in g:     # g in Pos^-1(i) over ALL users (sampler_gbpr.py:41)
                    assert i in ix[ip[gg]:ip[gg + 1]]
                    cross += int(not (u0 <= gg < u1))
    assert cross > 0
    assert np.array_equal(res[0][4], res[1][4]) and np.array_equal(res[0][5], res[1][5])


@pytest.mark.parametrize("exchange", ["allreduce", "rs_ag"])
def test_pipelined_count_exchange_equals_synchronous(fold1, exchange):
    """Device-sampled steps with the batch of step s+1 drawn, packed and its
    per-owner counts exchanged at the start of step s (cf_xchg_draw /
    cf_xchg_adopt: no host round trip inside the step) train exactly what the
    synchronous cf_xchg_begin path trains on the same sampler stream."""
    from oracle import cf_oracle as O
    rng = np.random.RandomState(14)
    d = 16
    U0 = O.init_table(rng, (943, d))
    V0 = O.init_table(rng, (1682, d))
    b0 = O.init_table(rng, (1682,))
    dummy = [(np.zeros((1, 2), np.int32), np.zeros((1, 5), np.int32), np.zeros((1, 1), np.int32))]
    a = _run(fold1, dummy, U0, V0, b0, sampled="steps", exchange=exchange, pipelined=True)
    b = _run(fold1, dummy, U0, V0, b0, sampled="steps", exchange=exchange, pipelined=False)
    for ra, rb in zip(a, b):
        for k in (3, 4, 5, 6):      # user, item, bias, acc_user
            assert_close(ra[k], rb[k], (ra[0], k))


@pytest.mark.parametrize("exchange", ["allreduce", "rs_ag"])
def test_pipelined_exchange_batch_size_change(fold1, exchange):
    """The batch drawn one step ahead is taken only at the size it was drawn
    at: when the caller changes batch_size between pipelined steps, the
    engine discards it (counts cleared, sampler rewound, CF_EAGAIN) and the
    step draws at the new size -- so the pipelined run trains exactly what
    the synchronous one trains over the same size sequence."""
    from oracle import cf_oracle as O
    rng = np.random.RandomState(15)
    d = 16
    U0 = O.init_table(rng, (943, d))
    V0 = O.init_table(rng, (1682, d))
    b0 = O.init_table(rng, (1682,))
    dummy = [(np.zeros((1, 2), np.int32), np.zeros((1, 5), np.int32), np.zeros((1, 1), np.int32))]
    a = _run(fold1, dummy, U0, V0, b0, sampled="sizes", exchange=exchange, pipelined=True)
    b = _run(fold1, dummy, U0, V0, b0, sampled="sizes", exchange=exchange, pipelined=False)
    for ra, rb in zip(a, b):
        for k in (3, 4, 5, 6, 8, 9):      # user, item, bias, acc_user, acc_item, acc_bias
            assert_close(ra[k], rb[k], (ra[0], k))
