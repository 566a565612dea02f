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
    """One data-parallel optimizer step: local phase -> all-reduce -> items."""

    def __init__(self, backend, item_grad, process_group=None):
        import torch.distributed as dist
        self.backend = backend
        self.item_grad = item_grad
        self.group = process_group
        self._dist = dist

    def __call__(self, batch_size=None, pairs=None, negs=None, groups=None):
        if pairs is None:
            self.backend.step_local(batch_size)
        else:
            self.backend.step_local(pairs=pairs, negs=negs, groups=groups)
        self._dist.all_reduce(self.item_grad, group=self.group)
        self.backend.step_items()


def make_gpu_sharded(engine, n_items, d, with_bias, device):
    """Bind a torch tensor as the engine's item-gradient buffer, run the
    engine on torch's current stream so RCCL orders after it, and return the
    step callable."""
    import torch
    n = n_items * d + (n_items if with_bias else 0)
    grad = torch.zeros(n, dtype=torch.float32, device=device)
    engine.set_stream(torch.cuda.current_stream(device).cuda_stream)
    engine.bind_item_grad(grad.data_ptr(), n)
    return ShardedStep(engine, grad), grad
