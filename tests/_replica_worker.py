"""Fold worker for the fold-parallel replica test (tests/test_gpu_models.py).

The same structure as the drivers' worker (testbprmf.py:32-52: text fold ->
loadSparseR -> matBinarize -> sampler -> BPRMF.train -> scores), but
deterministic so that each spawned replica can be compared with the oracle:
the reference sampler's own stream for np.random.seed(11) (ExactSampler) and
the seeded initial tables of tests/golden/make_cfg1_golden.py -- the cfg1
configuration whose oracle metrics are the committed fixture
tests/golden/cfg1_oracle_metrics.json.  Lives in its own module so that a
*spawned* child process can import it by name.
"""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cfg1_config():
    with open(os.path.join(GOLDEN, "cfg1_oracle_metrics.json")) as f:
        return json.load(f)


def seeded_worker(fold, n_users, n_items, dataset_dir):
    from collaborativefilteringusingtensorflow_amd.bprmf import BPRMF
    from collaborativefilteringusingtensorflow_amd.drivers._common import load_fold
    from collaborativefilteringusingtensorflow_amd.init_util import seeded_table
    from collaborativefilteringusingtensorflow_amd.sampler_ranking import ExactSampler
    c = cfg1_config()["config"]
    tra, tst = load_fold(dataset_dir, fold, n_users, n_items, 3)
    rng = np.random.RandomState(c["init_seed"])
    U0 = seeded_table(rng, (n_users, c["d"]))
    V0 = seeded_table(rng, (n_items, c["d"]))
    m = BPRMF(n_users, n_items, c["topN"], 'cv', c["metrics"], c["reg"], c["d"], c["B"],
              max_iter=c["epochs"], device=int(os.environ.get("CF_DEVICE", "0")), verbose=False)
    m.set_initial_tables(user=U0, item=V0)
    es = ExactSampler(tra, n_neg=c["W"], batch_size=c["B"], seed=c["sampler_seed"])
    scores = m.train(fold + 1, tra, tst, es)
    es.close()
    m.close()
    return [float(s) for s in scores]
