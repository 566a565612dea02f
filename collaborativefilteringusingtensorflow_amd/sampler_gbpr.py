"""Drop-in for ``src/samplers/sampler_gbpr.py``: ``Sampler(trasR, gsize=2,
n_neg=5, batch_size=100, n_workers=1).next_batch()`` returns
``(pairs [B,2] int32, negs [B,W] int64, groups [B,G] int64)``
(sampler_gbpr.py:43); each group user is drawn uniformly with replacement
from the positive item's users and may be u itself (sampler_gbpr.py:41).
Drawn on the GPU.
"""
import numpy as np

from ._sampler import DeviceSampler, MTSampler


class Sampler(DeviceSampler):
    def __init__(self, trasR, gsize=2, n_neg=5, batch_size=100, n_workers=1, seed=None,
                 device=0):
        if gsize < 1:
            raise ValueError("gsize must be >= 1")
        super(Sampler, self).__init__(trasR, n_neg=n_neg, batch_size=batch_size, gsize=gsize,
                                      n_workers=n_workers, seed=seed, device=device)

    def next_batch(self):
        pairs, negs, groups = self._draw()
        return pairs.astype(np.int32), negs.astype(np.int64), groups.astype(np.int64)


class ExactSampler(MTSampler):
    """Bit-exact host mode: the reference's stream for ``np.random.seed(seed)``
    (sampler_gbpr.py:23-43), same ``next_batch`` types."""
    KIND = 2

    def __init__(self, trasR, gsize=2, n_neg=5, batch_size=100, n_workers=1, seed=0):
        if gsize < 1:
            raise ValueError("gsize must be >= 1")
        super(ExactSampler, self).__init__(trasR, n_neg=n_neg, batch_size=batch_size,
                                           gsize=gsize, seed=seed)

    def next_batch(self):
        pairs, negs, groups = self._draw()
        return pairs, negs.astype(np.int64), groups.astype(np.int64)
