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


def assert_close(got, ref, what, rtol=RTOL, atol=ATOL, bound=None, max_excluded=0.0):
    """Elementwise |got - ref| <= atol + rtol |ref| (+ ``bound``, an a-priori
    fp32 bound from oracle/fp32_bound.py, where given) over the whole array.

    An element whose bound is not finite (inf, or NaN) checks nothing, so it
    fails the assertion -- unless the caller passes ``max_excluded``, the
    fraction of the touched elements (bound != 0) allowed to go unchecked;
    then those elements are excluded and their count is asserted.  Returns
    the worst |got - ref| / tol over the checked elements."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = np.abs(got - ref)
    tol = atol + rtol * np.abs(ref)
    if bound is not None:
        bound = np.asarray(bound, np.float64)
        fin = np.isfinite(bound)
        n_inf = int((~fin).sum())
        touched = int((bound != 0).sum())   # NaN != 0 and inf != 0: counted as touched
        assert n_inf <= max_excluded * touched, (
            "%s: %d of %d touched elements have a non-finite a-priori bound (allowed %.2g of them): "
            "they would go unchecked" % (what, n_inf, touched, max_excluded))
        if n_inf:
            got, ref, err, tol, bound = got[fin], ref[fin], err[fin], tol[fin], bound[fin]
        tol = tol + bound
    bad = err > tol
    worst = float(np.max(err / tol)) if err.size else 0.0
    if os.environ.get("CF_BAND_LOG"):   # margin survey: worst |d| / band per assertion
        with open(os.environ["CF_BAND_LOG"], "a") as f:
            f.write("%s\t%s\t%.4f\n" % (os.environ.get("PYTEST_CURRENT_TEST", "?"), what, worst))
    if bad.any():
        k = np.unravel_index(int(np.argmax(err / tol)), err.shape)
        raise AssertionError("%s: %d elements out of |d| <= %g + %g|ref|%s; worst d/bound %.3f at %s "
                             "(gpu %.9g, ref %.9g), max |d| %.3g"
                             % (what, int(bad.sum()), atol, rtol, " + E" if bound is not None else "",
                                worst, k, got[k], ref[k], float(err.max())))
    return worst


def assert_within(got, ref, bound, what):
    """|got - ref| <= bound elementwise, with bound the a-priori fp32 bound E
    of oracle/fp32_bound.py: E == 0 (a row the step does not touch) demands
    bit-identity.  Every E must be finite (a comparison with an infinite or
    NaN E is never false, so it would check nothing): callers exclude the
    rows they cannot bound and assert how many (LocalStepCheck)."""
    got = np.asarray(got, np.float64)
    assert np.isfinite(bound).all(), (what, int((~np.isfinite(bound)).sum()))
    err = np.abs(got - ref)
    bad = err > bound
    if bad.any():
        ratio = np.where(bound > 0, err / np.where(bound > 0, bound, 1.0), np.inf)
        k = np.unravel_index(int(np.argmax(ratio)), err.shape)
        raise AssertionError("%s: %d elements outside the a-priori fp32 bound; worst |d|/E %.3f at %s "
                             "(gpu %.9g, ref %.9g, E %.3g)"
                             % (what, int(bad.sum()), float(ratio[k]), k, got[k], ref[k], bound[k]))
    nz = bound > 0
    return float((err[nz] / bound[nz]).max()) if nz.any() else 0.0


BPR_TABLES = ("user", "item", "acc_user", "acc_item")


class LocalStepCheck:
    """Step-local parity of the BPR / AMF / CML step.

    Before each engine step, ``before(e)`` reads the engine's own float32
    tables; ``after(e, pairs, negs, loss)`` runs the float64 oracle one step
    from exactly those tables together with the a-priori fp32 bound E of
    oracle/fp32_bound.py, and requires every element of every table within E
    (untouched rows bit-identical) and the loss within 1e-5.  No constant in
    E is fitted to a GPU result; a hot row with one occurrence dropped or
    added twice lands 7-29x outside it (tests/test_fp32_bound.py).  CML: a
    pair within rounding of one of its branch thresholds (hinge, rank-weight
    indicators, argmin ties) may take either branch in fp32, so its rows are
    excluded (E = inf) -- at most ``max_excluded`` of the touched rows."""

    def __init__(self, reg=None, adversarial=None, reg_adv=1.0, model="bpr", max_excluded=0.01, **cml):
        self.model = model
        self.reg, self.adversarial, self.reg_adv = reg, adversarial, reg_adv
        self.cml = cml
        self.max_excluded = max_excluded
        self.worst = 0.0
        self.excluded = 0
        self.T = None

    def before(self, e):
        if self.T is None:
            self.T = {t: e.get_table(t) for t in BPR_TABLES}

    def after(self, e, pairs, negs, loss, what=""):
        from oracle import fp32_bound as FB
        L = {t: self.T[t].astype(np.float64) for t in BPR_TABLES}
        E = FB.zero_bounds(L["user"], L["item"], acc_exact=True)
        args = (L["user"], L["item"], L["acc_user"], L["acc_item"], E, np.asarray(pairs), np.asarray(negs))
        if self.model == "cml":
            lo = FB.cml_step_bounded(*args, **self.cml)
        else:
            lo = FB.bpr_step_bounded(*args, self.reg, adversarial=self.adversarial, reg_adv=self.reg_adv)
        assert abs(loss - lo) <= 1e-5 * abs(lo) + 1e-6, (what, loss, lo)
        self.T = {t: e.get_table(t) for t in BPR_TABLES}
        for t in BPR_TABLES:
            fin = np.isfinite(E[t])
            touched = (E[t] != 0).any(axis=1)
            bad_rows = (~fin).any(axis=1)
            self.excluded += int(bad_rows.sum())
            if self.model == "cml":   # only CML's branch-ambiguous pairs may go unbounded
                assert bad_rows.sum() <= max(2, self.max_excluded * touched.sum()), (what, t, int(bad_rows.sum()))
            else:                     # a one-step BPR / AMF bound is finite everywhere
                assert bad_rows.sum() == 0, (what, t, int(bad_rows.sum()))
            self.worst = max(self.worst, assert_within(self.T[t][~bad_rows], L[t][~bad_rows], E[t][~bad_rows],
                                                       "%s local %s" % (what, t)))
        log = os.environ.get("CF_BOUND_LOG")
        if log:   # the worst |gpu - oracle| / E so far, per test
            with open(log, "a") as f:
                f.write("%s %s %.4f %d\n" % (os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0], what,
                                            self.worst, self.excluded))
        return lo


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
