"""Device-backed samplers behind the reference's ``Sampler`` protocol.

The reference feeds every model from one producer thread per sampler
(src/samplers/sampler_ranking.py:8-40 and siblings): shuffle the nnz (u,i)
pairs each epoch, slice B-pair batches, draw W negatives per pair uniformly
and redraw while j is a positive of u, (GBPR) add G group users drawn with
replacement from the item's positive users.  Here the same stream is drawn by
the gfx950 sampler inside the engine (cf_sample / cf_train_steps): no thread,
no queue, no pickling, and no last-batch race.

When a model's ``train`` receives one of these samplers it does not pull
batches through ``next_batch`` at all: it runs the fused on-device
sample+step loop from the sampler's seed and position, and hands the position
back when done, so the stream continues where training left it.
"""
import ctypes
import os

import numpy as np

from . import _native as N
from .engine import Engine
from .io_util import to_csr


class DeviceSampler(object):
    _cf_device_sampler = True

    def __init__(self, trasR, n_neg=5, batch_size=100, gsize=0, n_workers=1, seed=None,
                 device=0):
        if batch_size < 1 or n_neg < 1:
            raise ValueError("batch_size and n_neg must be >= 1")
        self.indptr, self.indices, shape = to_csr(trasR)
        self.n_users, self.n_items = int(shape[0]), int(shape[1])
        self.batch_size, self.n_neg, self.gsize = int(batch_size), int(n_neg), int(gsize)
        self.n_workers = n_workers  # accepted for signature parity; the device needs no threads
        if seed is None:  # the reference never seeds
            seed = int.from_bytes(os.urandom(8), "little")
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.device = device
        self._engine = None
        self._state = (0, 0)

    def _eng(self):
        if self._engine is None:
            model = N.CF_GBPR if self.gsize > 0 else N.CF_BPR
            self._engine = Engine(model, self.n_users, self.n_items, 1, n_neg=self.n_neg,
                                  gsize=max(self.gsize, 1), device=self.device, seed=self.seed)
            self._engine.set_interactions(self.indptr, self.indices)
            self._engine.set_sampler_state(*self._state)
        return self._engine

    def state(self):
        return self._eng().sampler_state() if self._engine is not None else self._state

    def set_state(self, epoch, batch):
        self._state = (int(epoch), int(batch))
        if self._engine is not None:
            self._engine.set_sampler_state(epoch, batch)

    def _draw(self):
        return self._eng().sample(self.batch_size)

    def close(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None


def negatives_valid(indptr, indices, pairs, negs):
    """True iff no negative is a positive of its user (host-side check)."""
    for (u, _), js in zip(np.asarray(pairs), np.asarray(negs).reshape(len(pairs), -1)):
        row = indices[indptr[u]:indptr[u + 1]]
        if np.isin(js, row).any():
            return False
    return True


class MTSampler(object):
    """Bit-exact host mode (cf_mt_sampler): the batch
    stream the reference sampler produces after ``np.random.seed(seed)``,
    restated in C++ (numpy's legacy MT19937 shuffle / randint / choice).
    Models feed it host-side (cf_step), like any ``next_batch()`` object."""

    KIND = 0

    def __init__(self, trasR, n_neg=5, batch_size=100, gsize=0, seed=0):
        self.indptr, self.indices, shape = to_csr(trasR)
        self.n_users, self.n_items = int(shape[0]), int(shape[1])
        self.batch_size, self.n_neg, self.gsize = int(batch_size), int(n_neg), int(gsize)
        if not 0 <= int(seed) < 2 ** 32:
            raise ValueError("Seed must be between 0 and 2**32 - 1")  # np.random.seed's rule
        self._L = N.lib()
        self._h = ctypes.c_void_p()
        ip = np.ascontiguousarray(self.indptr, dtype=np.int64)
        ix = np.ascontiguousarray(self.indices, dtype=np.int32)
        N.check(self._L.cf_mt_sampler_create(ip.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                             ix.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                             self.n_users, self.n_items, self.KIND, self.n_neg,
                                             self.gsize, self.batch_size, int(seed),
                                             ctypes.byref(self._h)), "cf_mt_sampler_create")

    def _draw(self):
        B, W, G = self.batch_size, self.n_neg, self.gsize
        pairs = np.empty((B, 2), dtype=np.int32)
        negs = np.empty((B, W), dtype=np.int32)
        groups = np.empty((B, max(G, 1)), dtype=np.int32) if G else None
        P = ctypes.POINTER(ctypes.c_int32)
        N.check(self._L.cf_mt_sampler_next(self._h, pairs.ctypes.data_as(P), negs.ctypes.data_as(P),
                                           groups.ctypes.data_as(P) if G else None),
                "cf_mt_sampler_next")
        return pairs, negs, groups

    def state(self):
        e, b = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(self._L.cf_mt_sampler_state(self._h, ctypes.byref(e), ctypes.byref(b)),
                "cf_mt_sampler_state")
        return int(e.value), int(b.value)

    def close(self):
        if self._h:
            self._L.cf_mt_sampler_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
