"""A/B of the fused scoring + top-k pass at cfg5's shape (1M users x 100K items,
d = 128, top-10), on one GPU:

    python tools/score_ab.py [--users N] [--variants 0,3] [--no-exclude]

Builds bench.py's cfg5 engine (synthetic graph, AMF, a few training steps so
the tables are not at their init), then times score_topk over the users with
HIP events around the kernel (the engine's "topk" profile slot) for each
fused_variant, with and without the train-item exclusion.  Prints one JSON
line per case."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg5")
    ap.add_argument("--users", type=int, default=0, help="users scored (0 = all)")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--exclude", default="1,0", help="exclude_train settings to run")
    ap.add_argument("--train-steps", type=int, default=50)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--k", type=int, default=10)
    args = ap.parse_args()
    import bench
    from collaborativefilteringusingtensorflow_amd.engine import Engine, synth_graph
    from collaborativefilteringusingtensorflow_amd._native import KERNELS
    cfg = bench.CONFIGS[args.config]
    nu, ni, d = cfg["n_users"], cfg["n_items"], cfg["d"]
    indptr, indices = synth_graph(nu, ni, cfg["mean_degree"], cfg["zipf"], cfg["graph_seed"],
                                  n_threads=min(16, os.cpu_count() or 1))
    kw = {k: cfg[k] for k in ("margin", "reg_cov", "clip_norm", "reg_adv", "rho") if k in cfg}
    eng = Engine(cfg["model"], nu, ni, d, n_neg=cfg["W"], gsize=cfg["G"], reg=cfg["reg"], **kw)
    eng.set_interactions(indptr, indices)
    eng.init_params(0.0, 0.1, truncated=cfg["truncated"], seed=1)
    if cfg["model"] == "amf":
        eng.begin_phase(1)
    if args.train_steps:
        eng.train_steps(cfg["B"], args.train_steps, return_loss=False)
    eng.synchronize()
    n = args.users or nu
    users = np.arange(n, dtype=np.int32)
    flop = 2.0 * n * ni * d
    for v in [int(x) for x in args.variants.split(",")]:
        eng.set_option("fused_variant", v)
        for ex in [int(x) for x in args.exclude.split(",")]:
            eng.score_topk(users[:1024], args.k, exclude_train=bool(ex))   # warm-up
            eng.synchronize()
            best = None
            for _ in range(args.reps):
                eng.profile_reset()
                eng.set_option("profile_mask", 1 << KERNELS["topk"])
                eng.profile(True)
                t0 = time.perf_counter()
                eng.score_topk(users, args.k, exclude_train=bool(ex))
                eng.synchronize()
                wall = time.perf_counter() - t0
                eng.profile(False)
                ms, cnt = eng.profile_read("topk")
                r = {"variant": v, "exclude_train": ex, "users": n, "k": args.k,
                     "kernel_ms": ms, "kernel_TFLOPs": flop / (1e-3 * ms) / 1e12 if cnt and ms > 0 else None,
                     "wall_s": wall}
                if best is None or (r["kernel_ms"] < best["kernel_ms"]):
                    best = r
            print(json.dumps(best))
            sys.stdout.flush()


if __name__ == "__main__":
    main()
