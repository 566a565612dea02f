"""Drop-in for ``src/samplers/sampler_uij_ranking.py``: the W=1 variant whose
``next_batch()`` returns one ``[B,3]`` int64 array of (u, i, j) rows
(np.concatenate at sampler_uij_ranking.py:36).  Drawn on the GPU.
"""
import numpy as np

from ._sampler import DeviceSampler, MTSampler


class Sampler(DeviceSampler):
    def __init__(self, trasR, batch_size=100, n_workers=1, seed=None, device=0):
        super(Sampler, self).__init__(trasR, n_neg=1, batch_size=batch_size, gsize=0,
                                      n_workers=n_workers, seed=seed, device=device)

    def next_batch(self):
        pairs, negs, _ = self._draw()
        return np.concatenate((pairs, negs), axis=1).astype(np.int64)


class ExactSampler(MTSampler):
    """Bit-exact host mode: the reference's stream for ``np.random.seed(seed)``
    (sampler_uij_ranking.py:22-38), ``[B,3]`` int64 rows."""
    KIND = 1

    def __init__(self, trasR, batch_size=100, n_workers=1, seed=0):
        super(ExactSampler, self).__init__(trasR, n_neg=1, batch_size=batch_size, seed=seed)

    def next_batch(self):
        pairs, negs, _ = self._draw()
        return np.concatenate((pairs, negs), axis=1).astype(np.int64)
