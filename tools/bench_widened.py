"""Measurements of the SURVEY 8(f) rows beside the headline bench, on the GPU
box: the tuple models (PRIGP, CPLR), the Ensemble family, the bit-exact host
sampler, native ingest and fold-parallel replicas.  One JSON object on stdout.

    python tools/bench_widened.py > gpurun_out/widened.json

Inputs are the committed ml-100k fold-1 fixture (tests/golden/ml100k_fold1.npz)
and synthetic rating files written to a temp dir; every model runs at its
reference driver's settings (test*.py globals).  Rates are steady-state
(warm-up excluded, device synchronised on both sides of the timed loop).
"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from collaborativefilteringusingtensorflow_amd.init_util import seeded_table  # noqa: E402

NU, NI = 943, 1682


def fold1():
    z = np.load(os.path.join(ROOT, "tests", "golden", "ml100k_fold1.npz"))
    tra = sp.csr_matrix((np.ones(len(z["train_indices"]), np.float32), z["train_indices"],
                         z["train_indptr"]), shape=(NU, NI))
    tst = sp.csr_matrix((np.ones(len(z["test_indices"]), np.float32), z["test_indices"],
                         z["test_indptr"]), shape=(NU, NI))
    return z, sp.lil_matrix(tra), sp.lil_matrix(tst)


def timed(step, batches, warm=20):
    for b in batches[:warm]:
        step(b, False)
    t0 = time.perf_counter()
    for b in batches[warm:]:
        step(b, False)
    return t0


def ensemble_rates(tra):
    from collaborativefilteringusingtensorflow_amd.ensemble import EnsembleEngine
    from collaborativefilteringusingtensorflow_amd import sampler_uij_ranking, sampler_ranking
    out = {}
    rng = np.random.RandomState(0)
    cases = [("ensemble", 3, None, 0.01, 1.0, False),      # testensemble.py: K=3, reg=.01
             ("ensemble_", 5, 5, 0.1, 1.0, False),         # testensemble_.py: K=5, W=5
             ("ensemble__", 3, 5, 0.1, 0.1, True)]         # testensemble__.py: K=3, lambda=.1
    for name, K, W, reg, lam, singles in cases:
        e = EnsembleEngine(NU, NI, K, 100, reg=reg)
        for t, shape in (("user", (K, NU, 100)), ("item", (K, NI, 100)), ("h", (K, 100))):
            e.set_table(t, seeded_table(rng, shape))
        n = 420
        if W is None:
            s = sampler_uij_ranking.ExactSampler(tra, batch_size=100, seed=1)
            batches = [s.next_batch() for _ in range(n)]
            step = lambda b, rl: e.step(b, return_loss=rl)
        else:
            s = sampler_ranking.ExactSampler(tra, n_neg=W, batch_size=100, seed=1)
            batches = [s.next_batch() for _ in range(n)]
            step = lambda b, rl: e.step_w(b[0], b[1], lam=lam, singles=singles, return_loss=rl)
        s.close()
        t0 = timed(step, batches)
        e.take_loss()                                      # synchronises the stream
        dt = time.perf_counter() - t0
        steps = n - 20
        out[name] = {"K": K, "d": 100, "B": 100, "W": W or 1, "steps_per_s": steps / dt,
                     "triplets_per_s": steps * 100 * (W or 1) / dt,
                     "note": "host-fed steps at the reference driver's batch size (launch-bound)"}
        e.close()
    return out


def tuple_rates(tra):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    from collaborativefilteringusingtensorflow_amd._tuple import (PRIGPSampler, UITJSampler,
                                                                  coefficients, normalise_rows,
                                                                  top_k_rows, user_similarity)
    out = {}
    t0 = time.perf_counter()
    S = user_similarity(tra)
    prep_sim = time.perf_counter() - t0
    for name in ("prigp", "cplr"):
        t0 = time.perf_counter()
        if name == "prigp":     # testprigp.py: topK=5, alpha=10, reg=.1, d=100, B=1000
            coef = coefficients(top_k_rows(S.copy(), 5), tra, weighted=False)
            smp = PRIGPSampler(tra, coef, 1000, seed=3)
            e = Engine("prigp", NU, NI, 100, reg=0.1, alpha=10.0)
        else:                   # testcplr_u.py: topK=50, alpha=beta=gamma=1, reg=.01, d=100, B=1000
            coef = normalise_rows(coefficients(top_k_rows(S.copy(), 50, keep_short_rows=True), tra,
                                               weighted=True))
            smp = UITJSampler(tra, coef, 1000, seed=3)
            e = Engine("cplr", NU, NI, 100, reg=0.01)
        prep = time.perf_counter() - t0 + prep_sim
        e.init_params(0.0, 0.1, truncated=True, seed=5)
        n = 140
        t0 = time.perf_counter()
        batches = [smp.next_batch() for _ in range(n)]
        host_dt = time.perf_counter() - t0
        batches = [(b, None) if isinstance(b, np.ndarray) else b for b in batches]
        t1 = timed(lambda b, rl: e.step_plr(b[0], b[1], return_loss=rl), batches)
        e.take_loss()
        dt = time.perf_counter() - t1
        steps = n - 20
        out[name] = {"d": 100, "B": 1000, "tuples_per_s": steps * 1000 / dt,
                     "host_sampler_tuples_per_s": n * 1000 / host_dt,
                     "preprocess_s": prep,
                     "note": "engine step rate on pre-drawn tuples; host_sampler = the native "
                             "tuple sampler (cf_tuple_sampler, the Python loops' exact stream)"}
        e.close()
    return out


def sampler_rates(tra):
    from collaborativefilteringusingtensorflow_amd import sampler_ranking, sampler_gbpr
    out = {}
    for name, mk, W in (("sampler_ranking_b100_w1",
                         lambda: sampler_ranking.ExactSampler(tra, n_neg=1, batch_size=100, seed=1), 1),
                        ("sampler_ranking_b100_w5",
                         lambda: sampler_ranking.ExactSampler(tra, n_neg=5, batch_size=100, seed=1), 5),
                        ("sampler_gbpr_b100_g1_w5",
                         lambda: sampler_gbpr.ExactSampler(tra, 1, 5, 100, seed=1), 5)):
        s = mk()
        for _ in range(20):
            s.next_batch()
        n = 2000
        t0 = time.perf_counter()
        for _ in range(n):
            s.next_batch()
        dt = time.perf_counter() - t0
        s.close()
        out[name] = {"batches_per_s": n / dt, "triplets_per_s": n * 100 * W / dt,
                     "mode": "bit-exact numpy MT19937 stream, host, one thread"}
    return out


def ingest_rates(tmp):
    from collaborativefilteringusingtensorflow_amd.io_util import load_csr
    out = {}
    rng = np.random.RandomState(7)
    for name, lines, nu, ni in (("ml100k_fold_size", 80_000, NU, NI),
                                ("10M_lines", 10_000_000, 100_000, 50_000)):
        path = os.path.join(tmp, name + ".txt")
        u = rng.randint(0, nu, lines)
        i = rng.randint(0, ni, lines)
        r = rng.randint(1, 6, lines)
        with open(path, "w") as f:
            f.write("\n".join("%d\t%d\t%d" % t for t in zip(u.tolist(), i.tolist(), r.tolist())))
        mb = os.path.getsize(path) / 1e6
        load_csr(path, nu, ni, threshold=3)   # warm the page cache
        t0 = time.perf_counter()
        ip, ix = load_csr(path, nu, ni, threshold=3)[:2]
        dt = time.perf_counter() - t0
        out[name] = {"lines": lines, "MB": mb, "seconds": dt, "lines_per_s": lines / dt,
                     "MB_per_s": mb / dt, "nnz_after_binarize": int(ix.shape[0])}
        os.remove(path)
    return out


def fold_replicas(z, tmp):
    """5 folds of the testbprmf.py worker (50 epochs each) on the fixture fold,
    sequential vs one spawned process per fold (all on this box's device)."""
    from collaborativefilteringusingtensorflow_amd.drivers import _common, testbprmf
    ddir = os.path.join(tmp, "ml100k") + "/"
    os.makedirs(ddir, exist_ok=True)
    for k in range(5):
        for part in ("train", "test"):
            ip, ix = z[part + "_indptr"], z[part + "_indices"]
            users = np.repeat(np.arange(len(ip) - 1), np.diff(ip))
            with open(ddir + "ratings__%d_%s.txt" % (k + 1, "tra" if part == "train" else "tst"),
                      "w") as f:
                f.write("\n".join("%d\t%d\t5" % t for t in zip(users.tolist(), ix.tolist())))
    out = {}
    import contextlib
    import io
    for mode in ("sequential", "parallel"):
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            aves, stds = _common.run_folds(testbprmf.worker, NU, NI, ddir, 5, testbprmf.topN,
                                           testbprmf.eval_metrics, parallel=(mode == "parallel"),
                                           n_devices=1)
        out[mode] = {"seconds": time.perf_counter() - t0, "ndcg_ave": float(aves[-1])}
    out["note"] = "5 x (50 epochs of BPRMF d=100 on ml-100k fold 1), one GPU; parallel = 5 spawned processes"
    return out


def main():
    z, tra, _ = fold1()
    res = {"box": {"cpus_visible": os.cpu_count(), "omp_threads": os.environ.get("OMP_NUM_THREADS")}}
    with tempfile.TemporaryDirectory() as tmp:
        for key, fn in (("ensemble", lambda: ensemble_rates(tra)),
                        ("tuple_models", lambda: tuple_rates(tra)),
                        ("exact_sampler", lambda: sampler_rates(tra)),
                        ("ingest", lambda: ingest_rates(tmp)),
                        ("fold_replicas", lambda: fold_replicas(z, tmp))):
            t0 = time.perf_counter()
            res[key] = fn()
            print("%s done in %.1fs" % (key, time.perf_counter() - t0), file=sys.stderr)
            sys.stderr.flush()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
