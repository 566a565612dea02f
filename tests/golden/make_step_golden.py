"""Step goldens: the oracle's trajectory on the
reference's own captured batch streams, frozen as a small fixture.

Test infrastructure only; needs no reference code (the batch streams were
captured from the reference samplers by make_golden.py).  For each case: the
seeded initial tables (oracle.cf_oracle.init_table; truncated normal, normal
for CML), K oracle steps in float64 and in float32, and then

* the per-step pre-update loss (both precisions),
* fp64 checksums (sum, sum of squares) of every final table and accumulator,
* the final values of 24 touched user rows and 24 touched item rows
  (the first distinct ids of the stream) of every table,

so tests/test_step_golden.py can pin the oracle (CPU) and the engine (GPU)
to the same frozen numbers without shipping whole tables.

    python tests/golden/make_step_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import cf_oracle as O  # noqa: E402

NU, NI, K, NROWS = 943, 1682, 10, 24
# name, model, stream, d, hyper-parameters, AMF phase switch
CASES = [
    ("bpr", "bpr", "rank_b100_w1", 32, dict(reg=0.1), None),
    ("bpr_w5", "bpr", "rank_b100_w5", 16, dict(reg=0.05), None),
    ("gbpr", "gbpr", "gbpr_b100_g1_w5", 16, dict(reg=0.01, rho=0.4), None),
    ("gbpr_g3", "gbpr", "gbpr_b100_g3_w2", 16, dict(reg=0.02, rho=0.5), None),
    ("cml", "cml", "rank_b50_w5", 16, dict(margin=1.0, reg_cov=1.0, clip_norm=1.0), None),
    ("amf", "amf", "rank_b100_w5", 16, dict(reg=0.05, reg_adv=1.0), 5),
]


def init(model, d, dtype):
    rng = np.random.RandomState(20261016)
    trunc = model != "cml"
    U = O.init_table(rng, (NU, d), truncated=trunc).astype(dtype)
    V = O.init_table(rng, (NI, d), truncated=trunc).astype(dtype)
    b = O.init_table(rng, (NI,), truncated=trunc).astype(dtype) if model == "gbpr" else None
    return U, V, b


def run(model, st, d, hp, switch, dtype):
    U, V, b = init(model, d, dtype)
    AU, AV = np.full_like(U, 0.1), np.full_like(V, 0.1)
    Ab = np.full_like(b, 0.1) if b is not None else None
    losses = []
    for s in range(K):
        pr, ng = st["pairs"][s], st["negs"][s]
        if model == "bpr":
            lo = O.bpr_step(U, V, AU, AV, pr, ng, hp["reg"])
        elif model == "gbpr":
            lo = O.gbpr_step(U, V, b, AU, AV, Ab, pr, ng, st["groups"][s], hp["rho"], hp["reg"])
        elif model == "cml":
            lo = O.cml_step(U, V, AU, AV, pr, ng, hp["margin"], hp["reg_cov"], hp["clip_norm"])
        else:
            adv = switch is not None and s >= switch
            if adv and s == switch:
                AU[...] = 0.1
                AV[...] = 0.1
            lo = O.amf_step(U, V, AU, AV, pr, ng, hp["reg"], adv, reg_adv=hp["reg_adv"])
        losses.append(lo)
    tabs = {"user": U, "item": V, "acc_user": AU, "acc_item": AV}
    if b is not None:
        tabs.update(bias=b, acc_bias=Ab)
    return np.array(losses), tabs


def pick_rows(st):
    users = list(dict.fromkeys(st["pairs"][:K, :, 0].ravel().tolist()))[:NROWS]
    items = list(dict.fromkeys(np.concatenate([st["pairs"][:K, :, 1].ravel(),
                                               st["negs"][:K].ravel()]).tolist()))[:NROWS]
    return np.array(users, np.int32), np.array(items, np.int32)


def main():
    z = np.load(os.path.join(HERE, "sampler_streams.npz"))
    out = {}
    for name, model, stream, d, hp, switch in CASES:
        st = {k.split("/")[1]: z[k] for k in z.files if k.startswith(stream + "/")}
        ru, ri = pick_rows(st)
        out[name + "/rows_user"] = ru
        out[name + "/rows_item"] = ri
        for tag, dt in (("f64", np.float64), ("f32", np.float32)):
            losses, tabs = run(model, st, d, hp, switch, dt)
            out["%s/%s/loss" % (name, tag)] = losses
            for t, x in tabs.items():
                x64 = x.astype(np.float64)
                out["%s/%s/%s/checksum" % (name, tag, t)] = np.array([x64.sum(), (x64 * x64).sum()])
                rows = ru if t in ("user", "acc_user") else ri
                out["%s/%s/%s/rows" % (name, tag, t)] = x[rows]
    np.savez_compressed(os.path.join(HERE, "step_goldens.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
