import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT,):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built engine")
    config.addinivalue_line("markers", "slow: long-running")


# North-star tolerance on fp32 embeddings, elementwise: every element within
# |gpu - oracle| <= ATOL + RTOL |oracle| (ATOL covers elements that cancel to
# ~0 after an Adagrad update of ~0.1)
RTOL, ATOL = 1e-5, 1e-6
# CML trajectories: the oracle itself run in float32 -- the arithmetic width
# of TF1's CPU path -- leaves the strict band around the float64 oracle (the
# rank weight log(1 + n_items * ...) ~ 7 scales every gradient, the
# accumulators sum their squares) and stays inside this relaxed one
# (tests/test_oracle.py::test_fp32_oracle_drift_bounds_cml_tolerance)
CML_TRAJ = dict(rtol=5e-5, atol=3e-6)
# Ensemble stress shapes (tests/test_gpu_ensemble.py::test_ensemble_ragged_hot_rows:
# 50 x 80 tables, a hot user in a third of the pairs, the [B, B] cross loss of
# ensemble.py:84-91 summed into each row): the oracle run in float32 leaves
# the rtol 1e-4 band around the float64 oracle by up to 7.4x within six
# steps (an accumulator 2.9157 in float64 is 2.9132 in float32: sums of ~B^2
# cancelling terms per row), and stays under 0.5 of this one
# (tests/test_oracle.py::test_fp32_oracle_drift_bounds_ensemble_tolerance)
ENS_HOT = dict(rtol=2e-3, atol=1e-4)


def assert_close(got, ref, what, rtol=RTOL, atol=ATOL, ref32=None):
    """Elementwise |got - ref| <= atol + rtol |ref| over the whole array.
    With ref32 (the same oracle trajectory run in float32, the arithmetic
    width of TF1's CPU path) each element may also deviate by 3x the fp32
    oracle's own deviation from float64: a row that sums hundreds of
    cancelling gradient rows in fp32 (a Zipf-head item) moves by more than
    1e-5 relative in ANY fp32 summation order."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = np.abs(got - ref)
    bound = atol + rtol * np.abs(ref)
    if ref32 is not None:
        bound = bound + 3.0 * np.abs(np.asarray(ref32, np.float64) - ref)
    bad = err > bound
    worst = float(np.max(err / bound)) if err.size else 0.0
    if bad.any():
        k = np.unravel_index(int(np.argmax(err / bound)), err.shape)
        raise AssertionError("%s: %d elements out of |d| <= %g + %g|ref|; worst d/bound %.3f at %s "
                             "(gpu %.9g, ref %.9g), max |d| %.3g"
                             % (what, int(bad.sum()), atol, rtol, worst, k, got[k], ref[k], float(err.max())))
    return worst


@pytest.fixture(scope="session")
def fold1():
    z = np.load(os.path.join(GOLDEN, "ml100k_fold1.npz"))
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def streams():
    z = np.load(os.path.join(GOLDEN, "sampler_streams.npz"))
    return {k: z[k] for k in z.files}


def get_stream(streams, name):
    out = {"pairs": streams[name + "/pairs"], "negs": streams[name + "/negs"]}
    if name + "/groups" in streams:
        out["groups"] = streams[name + "/groups"]
    return out


@pytest.fixture(scope="session")
def gpu_available():
    try:
        from collaborativefilteringusingtensorflow_amd import _native as N
        return N.device_count() > 0
    except Exception:
        return False


@pytest.fixture(autouse=True)
def _require_gpu(request):
    if request.node.get_closest_marker("gpu") is not None:
        from collaborativefilteringusingtensorflow_amd import _native as N
        # fail loudly (not skip) when the native library is missing on a GPU run
        N.lib()
        if N.device_count() == 0:
            pytest.skip("no HIP device visible")
