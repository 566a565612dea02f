"""Frozen step goldens (tests/golden/step_goldens.npz, made by
tests/golden/make_step_golden.py from the reference's captured batch streams):
per-step losses, table checksums and touched rows after 10 steps of BPR (W=1,
W=5), GBPR (G=1, G=3), CML and AMF (across the phase switch).

* CPU: the oracle still reproduces them (1e-12 in float64, 1e-6 in float32),
  so a change to the oracle cannot silently move the parity target.
* GPU: the engine, fed the same batches from the same initial tables, lands
  on them within 1e-5 relative (fp32 device arithmetic vs the float64 golden).
"""
import os

import numpy as np
import pytest

from conftest import assert_close

HERE = os.path.dirname(os.path.abspath(__file__))
import sys  # noqa: E402
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_step_golden as G  # noqa: E402


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "step_goldens.npz"))
    return {k: z[k] for k in z.files}


def stream_of(streams, name):
    return {k.split("/")[1]: v for k, v in streams.items() if k.startswith(name + "/")}


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.parametrize("case", [c[0] for c in G.CASES])
@pytest.mark.parametrize("tag,dt,tol", [("f64", np.float64, 1e-12), ("f32", np.float32, 1e-6)])
def test_oracle_reproduces_step_golden(gold, streams, case, tag, dt, tol):
    name, model, stream, d, hp, switch = next(c for c in G.CASES if c[0] == case)
    losses, tabs = G.run(model, stream_of(streams, stream), d, hp, switch, dt)
    assert rel(losses, gold["%s/%s/loss" % (name, tag)]) <= tol
    for t, x in tabs.items():
        rows = gold[name + ("/rows_user" if t in ("user", "acc_user") else "/rows_item")]
        assert rel(x[rows], gold["%s/%s/%s/rows" % (name, tag, t)]) <= tol, t
        x64 = x.astype(np.float64)
        ck = gold["%s/%s/%s/checksum" % (name, tag, t)]
        assert abs(x64.sum() - ck[0]) <= tol * (abs(ck[0]) + ck[1]) + 1e-9, t
        assert abs((x64 * x64).sum() - ck[1]) <= tol * ck[1], t


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c[0] for c in G.CASES])
def test_engine_lands_on_step_golden(gold, streams, case):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    name, model, stream, d, hp, switch = next(c for c in G.CASES if c[0] == case)
    st = stream_of(streams, stream)
    W = st["negs"].shape[2]
    Gs = st["groups"].shape[2] if "groups" in st else 1
    kw = dict(hp)
    e = Engine(model, G.NU, G.NI, d, n_neg=W, gsize=Gs, **kw)
    U, V, b = G.init(model, d, np.float32)
    e.set_table("user", U)
    e.set_table("item", V)
    if b is not None:
        e.set_table("bias", b)
    losses = []
    for s in range(G.K):
        if switch is not None and s == switch:
            e.begin_phase(1)
        losses.append(e.step(st["pairs"][s], st["negs"][s], st.get("groups", [None] * G.K)[s]))
    assert rel(losses, gold["%s/f64/loss" % name]) <= 1e-5
    for t in ("user", "item", "acc_user", "acc_item") + (("bias", "acc_bias") if b is not None else ()):
        x = e.get_table(t)
        rows = gold[name + ("/rows_user" if t in ("user", "acc_user") else "/rows_item")]
        assert_close(x[rows], gold["%s/f64/%s/rows" % (name, t)], t)
        ck = gold["%s/f64/%s/checksum" % (name, t)]
        assert abs((x.astype(np.float64) ** 2).sum() - ck[1]) <= 1e-5 * ck[1], t
    e.close()


def test_seeded_table_is_the_oracle_init():
    """bench.py's cfg1 run and the cfg1 golden start from the same tables."""
    from collaborativefilteringusingtensorflow_amd.init_util import seeded_table
    from oracle import cf_oracle as O
    for trunc in (True, False):
        a = seeded_table(np.random.RandomState(11), (943, 32), truncated=trunc)
        b = O.init_table(np.random.RandomState(11), (943, 32), truncated=trunc)
        np.testing.assert_array_equal(a, b)
