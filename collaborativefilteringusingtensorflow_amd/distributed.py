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


def _gloo_dev(dist, t, group):
    """gloo stages device tensors through host copies (the collectives below
    are called on host copies and copied back)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


class _Works(object):
    def __init__(self, works):
        self.works = [w for w in works if w is not None]

    def wait(self):
        for w in self.works:
            w.wait()


class AllReduceItems(object):
    """Replicated item Adagrad: the dense item gradient (this rank's sum in
    ``grad``) is all-reduced, then every replica applies the identical update
    (``step_items``)."""

    name = "allreduce"
    draw_with_apply = True   # the next draw rides in the user-apply launch

    def __init__(self, grad, group=None, pieces=1, row_width=None, n_rows=None):
        self.grad = grad
        self.group = group
        # the item reduce in pieces of item rows (cf_step_item_reduce): piece
        # q's all-reduce is issued as soon as that piece is reduced, so it runs
        # while the next piece reduces; rows of row_width elements, then a
        # tail (GBPR's item bias) reduced with the last piece
        self.pieces = int(pieces)
        self.row_width = row_width
        self.n_rows = n_rows

    def overlap(self, dist):
        return self.grad.is_cuda and dist.get_backend(self.group) != "gloo"

    def reduce(self, dist, async_op, be=None):
        if self.pieces > 1 and be is not None and hasattr(be, "step_item_reduce"):
            w, works = self.row_width, []
            for q in range(self.pieces):
                be.step_item_reduce(q)
                r0, r1 = be.item_piece_rows(q, self.pieces)
                if r1 > r0:
                    works.append(dist.all_reduce(self.grad[r0 * w:r1 * w], group=self.group, async_op=async_op))
            if self.grad.numel() > self.n_rows * w:   # the bias tail
                works.append(dist.all_reduce(self.grad[self.n_rows * w:], group=self.group, async_op=async_op))
            return _Works(works if async_op else [])
        return dist.all_reduce(self.grad, group=self.group, async_op=async_op)

    def apply(self, be):
        be.step_items()

    def gather(self, dist, async_op):
        return None

    def sync_state(self, dist):
        return None


class ReduceScatterItems(object):
    """Item-range ownership.  The dense item gradient (padded to world * chunk
    rows) is reduce-scattered: rank r receives the cross-rank sum of rows
    [r*chunk, (r+1)*chunk), applies Adagrad to them alone
    (``step_items_range``) and the updated rows are all-gathered into every
    replica's table.  The same bytes cross xGMI as an all-reduce; the item
    Adagrad (and the accumulator rows it keeps current) is 1/world of the
    replicated one, and the user apply and the next draw each run beside one
    of the two collectives.  TF1's sum-before-update semantics are unchanged:
    every row's update sees the sum over the global batch.

    ``grad`` [world*chunk*d] (+ ``grad_bias`` [world*chunk], GBPR) are the
    bound gradient buffers, ``tables`` the (padded, flat) table storages to
    all-gather after the owner update as (tensor, row width) -- V and b --
    and ``state`` the accumulators gathered by ``sync_state``."""

    name = "rs_ag"
    draw_with_apply = False  # the next draw runs beside the all-gather

    def __init__(self, grad, grad_slice, tables, chunk, rank, grad_bias=None, bias_slice=None,
                 state=(), group=None, world=None):
        self.grad, self.grad_slice = grad, grad_slice
        self.grad_bias, self.bias_slice = grad_bias, bias_slice
        self.tables = list(tables)
        self.state = list(state)
        self.chunk, self.rank = int(chunk), int(rank)
        # world 1 owns every row: nothing goes stale (None: unknown, assume > 1)
        self.world = world
        self.row0, self.row1 = self.rank * self.chunk, (self.rank + 1) * self.chunk
        self.group = group
        # accumulators of rows other ranks own are stale after an owner
        # update until sync_state gathers them (Engine.get_table refuses them)
        self.stale = False
        self.stale_tables = ("acc_item", "acc_bias")

    def overlap(self, dist):
        return self.grad.is_cuda and dist.get_backend(self.group) != "gloo"

    def _rs(self, dist, out, inp, async_op):
        if _gloo_dev(dist, inp, self.group):
            o = out.cpu()
            dist.reduce_scatter_tensor(o, inp.cpu(), group=self.group)
            out.copy_(o)
            return None
        return dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=async_op)

    def _ag(self, dist, full, width, async_op):
        lo, hi = self.row0 * width, self.row1 * width
        if _gloo_dev(dist, full, self.group):
            f = full.cpu()
            dist.all_gather_into_tensor(f, f[lo:hi].clone(), group=self.group)
            full.copy_(f)
            return None
        # in place: this rank's chunk of the output is the input
        return dist.all_gather_into_tensor(full, full[lo:hi], group=self.group, async_op=async_op)

    def reduce(self, dist, async_op, be=None):
        w = [self._rs(dist, self.grad_slice, self.grad, async_op)]
        if self.grad_bias is not None:
            w.append(self._rs(dist, self.bias_slice, self.grad_bias, async_op))
        return _Works(w)

    def apply(self, be):
        # the full buffers are consumed: re-zero the touched rows for the next
        # step, then the owner's Adagrad on its rows
        be.clear_item_grad()
        be.step_items_range(self.row0, self.row1, self.grad_slice, self.bias_slice)
        self.stale = self.world != 1

    def gather(self, dist, async_op):
        return _Works([self._ag(dist, t, w, async_op) for t, w in self.tables])

    def sync_state(self, dist):
        """All-gather the owners' accumulator rows (checkpoint / inspection:
        only the owner keeps its range current during training)."""
        for t, w in self.state:
            self._ag(dist, t, w, False)
        self.stale = False


def _items(items, group):
    import torch
    return AllReduceItems(items, group) if torch.is_tensor(items) else items


class ShardedStep(object):
    """One data-parallel optimizer step: local phase -> item exchange -> items.

    ``items`` is the item exchange (``AllReduceItems`` / ``ReduceScatterItems``;
    a bare tensor means the all-reduce of that item-gradient tensor).  With a
    backend that splits the local phase (step_local_grad / step_local_apply,
    include/cf_engine.h) the exchange is issued as soon as the item gradient
    is complete and runs beside the user update and the draw of the next
    batch; the item update waits for it."""

    def __init__(self, backend, items, process_group=None, draw_ahead=True, apr_buf=None):
        import torch.distributed as dist
        self.backend = backend
        self.items = _items(items, process_group)
        self.item_grad = self.items.grad
        self.group = process_group
        self.draw_ahead = draw_ahead
        # AMF apr (include/cf_engine.h cf_step_local_apr_embed): the bound
        # [n_items * d] buffer of the embedding-loss sums, all-reduced before
        # the gradient launch in the adversarial phase
        self.apr_buf = apr_buf
        self._dist = dist

    def __call__(self, batch_size=None, pairs=None, negs=None, groups=None):
        be, x, dist = self.backend, self.items, self._dist
        if not hasattr(be, "step_local_grad"):
            if pairs is None:
                be.step_local(batch_size)
            else:
                be.step_local(pairs=pairs, negs=negs, groups=groups)
            x.reduce(dist, False)
            x.apply(be)
            x.gather(dist, False)
            return
        if self.apr_buf is not None and be.apr_active():
            # every item row's Δ from the global batch: this rank's sums, the
            # all-reduce, then the gradient launch on the summed buffer
            B = be.step_local_apr_embed(batch_size, pairs, negs)
            dist.all_reduce(self.apr_buf, group=self.group)
            be.step_local_grad(B)
        elif pairs is None:
            be.step_local_grad(batch_size)
        else:
            be.step_local_grad(pairs=pairs, negs=negs, groups=groups)
        # gloo stages device tensors through the host: overlap buys nothing
        # there (and its async device path serialises both ranks of a shared
        # GPU), so only RCCL gets the asynchronous collectives
        overlap = x.overlap(dist)
        nb = batch_size if (pairs is None and self.draw_ahead) else 0
        work = x.reduce(dist, overlap, be)
        be.step_local_apply(nb if x.draw_with_apply else 0)
        if overlap and work is not None:
            work.wait()
        x.apply(be)
        work = x.gather(dist, overlap)
        if nb and not x.draw_with_apply:
            be.step_local_draw(nb)
        if overlap and work is not None:
            work.wait()

    def sync_state(self):
        self.items.sync_state(self._dist)


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


def _bind_rs_items(engine, n_items, d, with_bias, device, group=None):
    """Padded torch buffers for item-range ownership, bound to the engine:
    gradient (+ bias gradient), the table storages V (+ b) the all-gather
    writes, and the accumulators (gathered by sync_state)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    chunk = -(-n_items // world)
    rows = world * chunk
    z = lambda n: torch.zeros(n, dtype=torch.float32, device=device)  # noqa: E731
    grad, gb = z(rows * d), (z(rows) if with_bias else None)
    engine.bind_item_grad_split(grad.data_ptr(), grad.numel(),
                                gb.data_ptr() if with_bias else None, rows if with_bias else 0)
    V, AV = z(rows * d), z(rows * d)
    engine.bind_table("item", V.data_ptr(), V.numel())
    engine.bind_table("acc_item", AV.data_ptr(), AV.numel())
    tables, state = [(V, d)], [(AV, d)]
    if with_bias:
        b, Ab = z(rows), z(rows)
        engine.bind_table("bias", b.data_ptr(), b.numel())
        engine.bind_table("acc_bias", Ab.data_ptr(), Ab.numel())
        tables.append((b, 1))
        state.append((Ab, 1))
    items = ReduceScatterItems(grad, z(chunk * d), tables, chunk, rank, grad_bias=gb,
                               bias_slice=z(chunk) if with_bias else None, state=state, group=group,
                               world=world)
    items._keep = (V, AV) + ((b, Ab) if with_bias else ())
    engine._stale_guard = items   # get_table refuses stale accumulators until sync_state
    return items


def make_gpu_sharded(engine, n_items, d, with_bias, device, exchange="allreduce", process_group=None,
                     pieces=1):
    """Bind the item-gradient buffer(s) to the engine, run the engine on
    torch's current stream so RCCL orders after it, and return the step
    callable and its item exchange.  ``exchange``: "allreduce" (dense
    all-reduce + replicated item Adagrad) or "rs_ag" (reduce-scatter ->
    owner Adagrad -> all-gather).  ``pieces`` > 1 (allreduce): the item
    reduce and its all-reduce in that many pieces of item rows."""
    import torch
    share_stream(engine, device)
    if exchange == "rs_ag":
        items = _bind_rs_items(engine, n_items, d, with_bias, device, process_group)
    elif exchange == "allreduce":
        n = n_items * d + (n_items if with_bias else 0)
        grad = torch.zeros(n, dtype=torch.float32, device=device)
        engine.bind_item_grad(grad.data_ptr(), n)
        if pieces > 1:
            engine.set_option("item_pieces", pieces)
        items = AllReduceItems(grad, process_group, pieces=pieces, row_width=d, n_rows=n_items)
    else:
        raise ValueError("exchange must be 'allreduce' or 'rs_ag'")
    apr_buf = None
    if getattr(engine, "cfg", None) is not None and engine.cfg.amf_mode == 1:   # CF_AMF_APR
        apr_buf = torch.zeros(n_items * d, dtype=torch.float32, device=device)
        engine.bind_apr_item_grad(apr_buf.data_ptr(), apr_buf.numel())
    return ShardedStep(engine, items, process_group, apr_buf=apr_buf), items


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


def _a2a(dist, out, inp, out_splits, in_splits, group, async_op=False):
    """all_to_all_single along dim 0; gloo gets host copies of device tensors
    (synchronously).  With ``async_op`` on RCCL the work handle is returned
    (the collective runs beside later launches on the stream until waited);
    otherwise None once complete."""
    if out.is_cuda and dist.get_backend(group) == "gloo":
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
        return None
    w = dist.all_to_all_single(out, inp, out_splits, in_splits, group=group, async_op=async_op)
    return w if async_op else None


class GroupExchangeStep(object):
    """One data-parallel GBPR step with the cross-shard group exchange.

    ``backend`` provides xchg_begin / xchg_serve / xchg_grad / xchg_finish /
    step_items (the C-ABI protocol in include/cf_engine.h), the exchange
    tensors send_ids, rows, grads, recv_ids, serve_rows, serve_grads,
    ``ensure_recv(n)`` and ``device``.

    Device-sampled steps (``batch_size``, no host batch) on a backend with
    ``xchg_draw`` / ``xchg_adopt`` are pipelined so that no step waits on the
    host: the batch of step s+1 is drawn and packed, its per-owner counts
    all-to-all'ed and copied to pinned host memory at the START of step s
    (before step s's exchange work in stream order); step s+1 then only waits
    on that copy's event, long complete, for the split sizes of its
    all-to-alls."""

    def __init__(self, backend, items, world, process_group=None, pipelined=True, split=True):
        import torch
        import torch.distributed as dist
        self.split = split
        self.backend = backend
        self.items = _items(items, process_group)
        self.item_grad = self.items.grad
        self.world = world
        self.group = process_group
        self._dist = dist
        self._torch = torch
        self.pipelined = pipelined and hasattr(backend, "xchg_draw")
        self._next = None
        if self.pipelined:
            dev = backend.device
            self._sc = torch.zeros((2, world), dtype=torch.int32, device=dev)
            self._rc = torch.zeros((2, world), dtype=torch.int32, device=dev)
            pin = dev.type == "cuda"
            self._hsc = torch.zeros((2, world), dtype=torch.int32, pin_memory=pin)
            self._hrc = torch.zeros((2, world), dtype=torch.int32, pin_memory=pin)

    def _draw(self, batch_size):
        torch = self._torch
        h = self.backend.xchg_draw(batch_size, self._sc.data_ptr())
        _a2a(self._dist, self._rc[h], self._sc[h], None, None, self.group)
        self._hsc[h].copy_(self._sc[h], non_blocking=True)
        self._hrc[h].copy_(self._rc[h], non_blocking=True)
        ev = torch.cuda.Event() if self._sc.is_cuda else None
        if ev is not None:
            ev.record()
        self._next = (h, ev)

    def _counts(self, batch_size, pairs, negs, groups):
        """(send counts, recv counts, send_ids half) of this step."""
        be, dist, torch = self.backend, self._dist, self._torch
        if self.pipelined and pairs is None:
            # the batch drawn one step ahead is adopted only at the size it
            # was drawn at; dropped by another call or drawn at another size
            # (the engine then discards it: counts cleared, sampler rewound),
            # it is drawn again now
            if self._next is not None and not be.xchg_adopt(batch_size):
                self._next = None
            if self._next is None:
                self._draw(batch_size)
                if not be.xchg_adopt(batch_size):
                    raise RuntimeError("cf_xchg_adopt refused the batch just drawn")
            h, ev = self._next
            if ev is not None:
                ev.synchronize()           # recorded a step ago: already complete
            sc, rc = self._hsc[h].tolist(), self._hrc[h].tolist()
            self._next = None
            self._draw(batch_size)         # step s+1, ahead of this step's exchange
            return sc, rc, h
        self._next = None
        sc = be.xchg_begin(self.world, batch_size=batch_size, pairs=pairs, negs=negs, groups=groups)
        sct = torch.as_tensor(np.asarray(sc, dtype=np.int64)).to(be.device)
        rct = torch.empty_like(sct)
        _a2a(dist, rct, sct, None, None, self.group)
        return [int(x) for x in sc], [int(x) for x in rct.tolist()], 0

    def __call__(self, batch_size=None, pairs=None, negs=None, groups=None):
        be, dist = self.backend, self._dist
        sc, rc, h = self._counts(batch_size, pairs, negs, groups)
        ns, nr = sum(sc), sum(rc)
        be.ensure_recv(nr)
        cap = getattr(be, "send_cap", 0)
        _a2a(dist, be.recv_ids[:nr], be.send_ids[h * cap:h * cap + ns], rc, sc, self.group)
        be.xchg_serve(nr)
        x = self.items
        # one rank has no remote members to overlap with (the split only adds
        # a launch and an apply there); a rank with none to fetch (ns == 0)
        # runs its whole gradient at once beside the rows it serves.
        # split == "force" takes the split step (both gradient parts, the
        # asynchronous collectives) at any world size -- the one-rank RCCL
        # test of its stream ordering (tests/test_gpu_group_exchange.py)
        force = self.split == "force"
        if not (self.split and (self.world > 1 or force) and hasattr(be, "xchg_grad_part")):
            _a2a(dist, be.rows[:ns], be.serve_rows[:nr], sc, rc, self.group)
            be.xchg_grad()
            _a2a(dist, be.serve_grads[:nr], be.grads[:ns], rc, sc, self.group)
            be.xchg_finish(nr)
            x.reduce(dist, False)
            x.apply(be)
            x.gather(dist, False)
            return
        # split step: the pairs whose members are all local run while the
        # member rows are in flight, the items' sums start the item exchange
        # while the member gradients are in flight; the user update waits for
        # them (exact sum-before-update, gbprmf.py:101-106)
        overlap = x.overlap(dist)
        w = _a2a(dist, be.rows[:ns], be.serve_rows[:nr], sc, rc, self.group, async_op=overlap)
        if ns > 0 or force:
            be.xchg_grad_part(1)
            if w is not None:
                w.wait()
            be.xchg_grad_part(2)
        else:
            be.xchg_grad()
            if w is not None:
                w.wait()
        w = _a2a(dist, be.serve_grads[:nr], be.grads[:ns], rc, sc, self.group, async_op=overlap)
        be.xchg_finish_items()
        work = x.reduce(dist, overlap)
        if w is not None:
            w.wait()
        be.xchg_finish(nr)
        if overlap and work is not None:
            work.wait()
        x.apply(be)
        work = x.gather(dist, overlap)
        if overlap and work is not None:
            work.wait()

    def sync_state(self):
        self.items.sync_state(self._dist)


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
        # two halves: the batch drawn one step ahead packs into the other one
        self.send_ids = torch.empty(2 * cap, dtype=torch.int32, device=device)
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

    def xchg_draw(self, batch_size, counts_ptr):
        return self.e.xchg_draw(batch_size, counts_ptr)

    def xchg_adopt(self, batch_size):
        return self.e.xchg_adopt(batch_size)

    def xchg_serve(self, n):
        self.e.xchg_serve(n)

    def xchg_grad(self):
        self.e.xchg_grad()

    def xchg_grad_part(self, part):
        self.e.xchg_grad_part(part)

    def xchg_finish_items(self):
        self.e.xchg_finish_items()

    def xchg_finish(self, n):
        self.e.xchg_finish(n)

    def step_items(self):
        self.e.step_items()

    def clear_item_grad(self):
        self.e.clear_item_grad()

    def step_items_range(self, row0, row1, grad, grad_bias=None):
        self.e.step_items_range(row0, row1, grad, grad_bias)


def make_gpu_group_exchange(engine, world, rank, bounds, indptr, indices, n_items, d, batch_size,
                            device, process_group=None, exchange="allreduce", item_csr=None):
    """Sharded GBPR on the real engine: bind the item-gradient buffers and the
    exchange buffers, run on torch's current stream (RCCL orders after the
    engine's kernels), return the step callable and its item exchange.
    ``indptr``/``indices`` are the GLOBAL user -> item CSR, or pass the global
    item -> user CSR directly as ``item_csr`` = (indptr_t, indices_t)."""
    import torch
    share_stream(engine, device)
    if exchange == "rs_ag":
        items = _bind_rs_items(engine, n_items, d, True, device, process_group)
    elif exchange == "allreduce":
        n = n_items * d + n_items
        grad = torch.zeros(n, dtype=torch.float32, device=device)
        engine.bind_item_grad(grad.data_ptr(), n)
        items = AllReduceItems(grad, process_group)
    else:
        raise ValueError("exchange must be 'allreduce' or 'rs_ag'")
    ip_t, ix_t = item_csr if item_csr is not None else item_users(indptr, indices, n_items)
    be = EngineExchange(engine, world, rank, bounds, ip_t, ix_t, batch_size, d, device)
    return GroupExchangeStep(be, items, world, process_group), items
