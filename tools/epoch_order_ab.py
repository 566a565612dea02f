"""A/B of the sorted batches' epoch order on the cfg2 graph (1M x 100K,
50M pairs): the counting scatter (cf_set_option "epoch_sort" 0, cf_epoch.hip)
against the hipCUB radix sort (1), records and index form, at B = 2^19 and
65,536.  Each order is computed in line on the engine stream (a sampler-state
jump to an uncached epoch, one sample), timed with the engine's HIP events.

    python tools/epoch_order_ab.py [--reps 5]   (run it under rocprofv3 for
    the per-kernel split)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    args = ap.parse_args()
    from collaborativefilteringusingtensorflow_amd import _native as N
    from collaborativefilteringusingtensorflow_amd.engine import Engine, synth_graph
    ip, ix = synth_graph(args.users, args.items, 50.0, 0.8, 20261015, n_threads=16)
    out = {"nnz": int(len(ix))}
    for sb in (1, 3):
        for B in (1 << 19, 65536):
            for es in (0, 1):
                e = Engine("bpr", args.users, args.items, 8, n_neg=1, seed=1)
                e.set_option("sorted_batches", sb)
                e.set_option("epoch_sort", es)
                e.set_interactions(ip, ix)
                e.sample(B)   # allocate, first order
                e.synchronize()
                e.profile_reset()
                e.set_option("profile_mask", 1 << N.KERNELS["epoch_order"])
                ms = []
                for r in range(args.reps):
                    e.profile_reset()
                    e.profile(True)
                    e.set_sampler_state(100 + 10 * r, 0)
                    e.sample(B)
                    e.synchronize()
                    e.profile(False)
                    t, n = e.profile_read("epoch_order")
                    ms.append(t / max(n, 1))
                key = "%s_B%d_%s" % ("records" if sb == 1 else "index", B, "count" if es == 0 else "radix")
                out[key] = {"ms_min": min(ms), "ms_med": sorted(ms)[len(ms) // 2]}
                print(key, out[key], flush=True)
                e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
