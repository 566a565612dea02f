"""User-sharded data parallelism over torch.distributed (RCCL on ROCm).

The reference has no multi-device path (fold-level multiprocessing only,
testbprmf.py:113-125).  This is the MI355X-native data-parallel layout of the
same optimizer step:

* users are partitioned into contiguous id ranges balanced by interaction
  count; each rank owns U, its Adagrad accumulator and the CSR rows of its
  users, and samples only its own pairs (negatives range over all items);
* item rows V (and GBPR's b) and their accumulators are replicated;
* per step every rank runs the local phase (sample, gather, loss, gradient
  scatter, user Adagrad -- exact, users are rank-exclusive), the dense fp32
  item gradient is all-reduced (sum), and every replica applies the identical
  item Adagrad.  Because TF1 sums duplicate rows over the whole batch before
  the update, this equals one step on the concatenation of the ranks' batches
  (up to fp32 summation order).

``ShardedStep`` only needs a backend with ``step_local(...)``, ``step_items()``
and an ``item_grad`` tensor; on GPU that is a native ``Engine`` whose item
gradient lives in a torch tensor, and the CPU tests drive the same class with
gloo and an oracle-backed stand-in.

GBPR draws each pair's group members from ALL users who consumed the item
(``item_posUserList``, sampler_gbpr.py:15,41), so on a user-sharded engine a
member may live on another rank.  ``GroupExchangeStep`` adds the exchange:
the ids of remote members go to their owners (all-to-all), the owners answer
with the pre-update rows (all-to-all), the gradient rows of those members go
back (all-to-all) and are summed with the owner's own contributions before
its Adagrad update -- still exactly one step on the concatenated batch.
"""
import numpy as np


def shard_users(indptr, world, rank):
    """Contiguous user range [u0, u1) of ``rank`` balancing nnz across ranks."""
    indptr = np.asarray(indptr, dtype=np.int64)
    n_users = indptr.shape[0] - 1
    nnz = int(indptr[-1])
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(indptr, nnz * r // world, side="left")))
    cuts.append(n_users)
    cuts = np.maximum.accumulate(np.minimum(np.asarray(cuts), n_users))
    return int(cuts[rank]), int(cuts[rank + 1])


def local_csr(indptr, indices, u0, u1):
    """CSR rows [u0, u1) rebased to local user ids."""
    indptr = np.asarray(indptr, dtype=np.int64)
    lo, hi = indptr[u0], indptr[u1]
    return (indptr[u0:u1 + 1] - lo).astype(np.int64), np.asarray(indices[lo:hi], dtype=np.int32)


class ShardedStep(object):
    """One data-parallel optimizer step: local phase -> all-reduce -> items.

    With a backend that splits the local phase (step_local_grad /
    step_local_apply, include/cf_engine.h) the all-reduce is issued as soon
    as the item gradient is complete and runs beside the user update and the
    draw of the next batch; the item update waits for it."""

    def __init__(self, backend, item_grad, process_group=None, draw_ahead=True):
        import torch.distributed as dist
        self.backend = backend
        self.item_grad = item_grad
        self.group = process_group
        self.draw_ahead = draw_ahead
        self._dist = dist

    def __call__(self, batch_size=None, pairs=None, negs=None, groups=None):
        be = self.backend
        if not hasattr(be, "step_local_grad"):
            if pairs is None:
                be.step_local(batch_size)
            else:
                be.step_local(pairs=pairs, negs=negs, groups=groups)
            self._dist.all_reduce(self.item_grad, group=self.group)
            be.step_items()
            return
        if pairs is None:
            be.step_local_grad(batch_size)
        else:
            be.step_local_grad(pairs=pairs, negs=negs, groups=groups)
        # gloo stages device tensors through the host: overlap buys nothing
        # there (and its async device path serialises both ranks of a shared
        # GPU), so only RCCL gets the asynchronous all-reduce
        overlap = self.item_grad.is_cuda and self._dist.get_backend(self.group) != "gloo"
        work = self._dist.all_reduce(self.item_grad, group=self.group, async_op=overlap)
        be.step_local_apply(batch_size if (pairs is None and self.draw_ahead) else 0)
        if overlap:
            work.wait()
        be.step_items()


def share_stream(engine, device):
    """Run the engine and torch (RCCL collectives, copies) on ONE stream so
    collectives order after the engine's kernels.  torch's default stream has
    handle 0, which the C ABI reads as "the engine's own stream", so a
    dedicated stream is made torch's current stream for this device."""
    import torch
    cur = torch.cuda.current_stream(device)
    if cur.cuda_stream == 0:
        cur = torch.cuda.Stream(device)
        torch.cuda.set_stream(cur)
    engine.set_stream(cur.cuda_stream)
    return cur


def make_gpu_sharded(engine, n_items, d, with_bias, device):
    """Bind a torch tensor as the engine's item-gradient buffer, run the
    engine on torch's current stream so RCCL orders after it, and return the
    step callable."""
    import torch
    n = n_items * d + (n_items if with_bias else 0)
    share_stream(engine, device)
    grad = torch.zeros(n, dtype=torch.float32, device=device)
    engine.bind_item_grad(grad.data_ptr(), n)
    return ShardedStep(engine, grad), grad


def item_users(indptr, indices, n_items):
    """Global item -> user CSR (the transpose of the user -> item CSR), the
    group source of a sharded GBPR engine (item_posUserList)."""
    indptr = np.asarray(indptr, dtype=np.int64)
    indices = np.asarray(indices, dtype=np.int64)
    users = np.repeat(np.arange(indptr.shape[0] - 1, dtype=np.int64), np.diff(indptr))
    order = np.argsort(indices, kind="stable")
    tp = np.zeros(n_items + 1, dtype=np.int64)
    np.add.at(tp, indices + 1, 1)
    return np.cumsum(tp), users[order].astype(np.int32)


def _a2a(dist, out, inp, out_splits, in_splits, group):
    """all_to_all_single along dim 0; gloo gets host copies of device tensors."""
    if out.is_cuda and dist.get_backend(group) == "gloo":
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


class GroupExchangeStep(object):
    """One data-parallel GBPR step with the cross-shard group exchange.

    ``backend`` provides xchg_begin / xchg_serve / xchg_grad / xchg_finish /
    step_items (the C-ABI protocol in include/cf_engine.h), the exchange
    tensors send_ids, rows, grads, recv_ids, serve_rows, serve_grads,
    ``ensure_recv(n)`` and ``device``."""

    def __init__(self, backend, item_grad, world, process_group=None):
        import torch
        import torch.distributed as dist
        self.backend = backend
        self.item_grad = item_grad
        self.world = world
        self.group = process_group
        self._dist = dist
        self._torch = torch

    def __call__(self, batch_size=None, pairs=None, negs=None, groups=None):
        be, dist, torch = self.backend, self._dist, self._torch
        sc = be.xchg_begin(self.world, batch_size=batch_size, pairs=pairs, negs=negs, groups=groups)
        sct = torch.as_tensor(np.asarray(sc, dtype=np.int64)).to(be.device)
        rct = torch.empty_like(sct)
        _a2a(dist, rct, sct, None, None, self.group)
        sc = [int(x) for x in sc]
        rc = [int(x) for x in rct.tolist()]
        ns, nr = sum(sc), sum(rc)
        be.ensure_recv(nr)
        _a2a(dist, be.recv_ids[:nr], be.send_ids[:ns], rc, sc, self.group)
        be.xchg_serve(nr)
        _a2a(dist, be.rows[:ns], be.serve_rows[:nr], sc, rc, self.group)
        be.xchg_grad()
        _a2a(dist, be.serve_grads[:nr], be.grads[:ns], rc, sc, self.group)
        be.xchg_finish(nr)
        dist.all_reduce(self.item_grad, group=self.group)
        be.step_items()


class EngineExchange(object):
    """GPU backend of GroupExchangeStep: a native GBPR Engine (user-sharded,
    dense item apply) with torch-owned exchange buffers bound to it."""

    def __init__(self, engine, world, rank, bounds, indptr_t, indices_t, batch_size, d, device):
        import torch
        self.e = engine
        self.d = d
        self.device = device
        self._torch = torch
        engine.set_shard(world, rank, bounds)
        engine.set_group_source(indptr_t, indices_t)
        cap = int(batch_size) * int(engine.gsize)
        self.send_ids = torch.empty(cap, dtype=torch.int32, device=device)
        self.rows = torch.empty((cap, d), dtype=torch.float32, device=device)
        self.grads = torch.empty((cap, d), dtype=torch.float32, device=device)
        self.send_cap = cap
        self._alloc_recv(max(1, cap * (world - 1)))

    def _alloc_recv(self, n):
        torch = self._torch
        self.recv_ids = torch.empty(n, dtype=torch.int32, device=self.device)
        self.serve_rows = torch.empty((n, self.d), dtype=torch.float32, device=self.device)
        self.serve_grads = torch.empty((n, self.d), dtype=torch.float32, device=self.device)
        self.recv_cap = n
        self.e.bind_exchange(self.send_ids.data_ptr(), self.rows.data_ptr(), self.grads.data_ptr(),
                             self.send_cap, self.recv_ids.data_ptr(), self.serve_rows.data_ptr(),
                             self.serve_grads.data_ptr(), self.recv_cap)

    def ensure_recv(self, n):
        if n > self.recv_cap:
            self._alloc_recv(n)

    def xchg_begin(self, world, **kw):
        return self.e.xchg_begin(world, **kw)

    def xchg_serve(self, n):
        self.e.xchg_serve(n)

    def xchg_grad(self):
        self.e.xchg_grad()

    def xchg_finish(self, n):
        self.e.xchg_finish(n)

    def step_items(self):
        self.e.step_items()


def make_gpu_group_exchange(engine, world, rank, bounds, indptr, indices, n_items, d, batch_size,
                            device, process_group=None):
    """Sharded GBPR on the real engine: bind the item-gradient tensor and the
    exchange buffers, run on torch's current stream (RCCL orders after the
    engine's kernels), return the step callable and the item-gradient tensor.
    ``indptr``/``indices`` are the GLOBAL user -> item CSR."""
    import torch
    n = n_items * d + n_items
    share_stream(engine, device)
    grad = torch.zeros(n, dtype=torch.float32, device=device)
    engine.bind_item_grad(grad.data_ptr(), n)
    ip_t, ix_t = item_users(indptr, indices, n_items)
    be = EngineExchange(engine, world, rank, bounds, ip_t, ix_t, batch_size, d, device)
    return GroupExchangeStep(be, grad, world, process_group), grad
