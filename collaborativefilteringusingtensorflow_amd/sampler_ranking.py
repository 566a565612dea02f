"""Drop-in for ``src/samplers/sampler_ranking.py`` (the sampler that actually
feeds BPRMF, CML and AMF: testbprmf.py:13, testcml.py:12, testamf.py:13).

``Sampler(trasR, n_neg=5, batch_size=100, n_workers=1).next_batch()`` returns
``(pairs [B,2] int32, negs [B,W] int64)`` like the reference
(sampler_ranking.py:37); batches are drawn on the GPU.
"""
import numpy as np

from ._sampler import DeviceSampler, MTSampler


class Sampler(DeviceSampler):
    def __init__(self, trasR, n_neg=5, batch_size=100, n_workers=1, seed=None, device=0):
        super(Sampler, self).__init__(trasR, n_neg=n_neg, batch_size=batch_size, gsize=0,
                                      n_workers=n_workers, seed=seed, device=device)

    def next_batch(self):
        pairs, negs, _ = self._draw()
        return pairs.astype(np.int32), negs.astype(np.int64)


class ExactSampler(MTSampler):
    """Bit-exact host mode: the reference's stream for ``np.random.seed(seed)``
    (sampler_ranking.py:22-37), same ``next_batch`` types."""
    KIND = 0

    def __init__(self, trasR, n_neg=5, batch_size=100, n_workers=1, seed=0):
        super(ExactSampler, self).__init__(trasR, n_neg=n_neg, batch_size=batch_size, seed=seed)

    def next_batch(self):
        pairs, negs, _ = self._draw()
        return pairs, negs.astype(np.int64)
