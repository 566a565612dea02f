"""Seeded initial tables for reproducible runs.

The reference initialises with TF's unseeded truncated_normal / random_normal
(bprmf.py:29-34, cml.py:32-37); a run that must be compared number for number
(cfg1's NDCG@10 against the oracle, bench.py) starts instead from this seeded
numpy draw and hands it to ``set_initial_tables``: standard normals, each one
beyond two standard deviations redrawn (truncated), scaled by stddev.
"""
import numpy as np


def seeded_table(rng, shape, stddev=0.1, truncated=True, dtype=np.float32):
    x = rng.standard_normal(size=shape)
    if truncated:
        bad = np.abs(x) > 2.0
        while bad.any():
            x[bad] = rng.standard_normal(size=int(bad.sum()))
            bad = np.abs(x) > 2.0
    return (x * stddev).astype(dtype)
