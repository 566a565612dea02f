"""Summarise rocprofv3 PMC passes into profiles/pmc_traffic.json.

    python tools/pmc_summary.py <tag> <fetch_dir> <write_dir> [trace_dir]

HBM bytes per launch, per kernel, from the TCC counters as
MI355X_MICROARCH.md prescribes: FETCH_SIZE and WRITE_SIZE come from separate
passes (they cannot share the TCC slots); both are in KiB; on gfx950
FETCH_SIZE reports exactly half of the bytes of a WIDE COALESCED streaming
read, so ``fetch_bytes_corrected = 2 * FETCH_SIZE * 1024`` is reported next
to the raw value (our row gathers are 64-B segments per 16-lane group, an
access width the guide lists as uncalibrated -- see DESIGN.md).  Infinity
Cache hits are counted by these counters, not excluded.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = {"grad_fast_kernel": "step", "grad_sort_kernel": "step", "grad_lds_kernel": "step", "grad_kernel": "step",
         "apply_prep_kernel": "apply_prep", "fused_topk_pipe_kernel": "fused_topk",
         "apply_ps_kernel<1, true": "apply_prep", "apply_ps_kernel<2, true": "apply_prep",
         "apply_ps_kernel<4, true": "apply_prep", "apply_ps_kernel<8, true": "apply_prep",
         "apply_ps_kernel": "apply", "psort_tile_sum_kernel": "psort_scan", "psort_tile_scan_kernel": "psort_scan",
         "prep_kernel": "sample", "slot_kernel": "slot", "apply_kernel": "apply",
         "apply_dense_kernel": "apply_dense", "clip_full_kernel": "clip",
         "fused_topk_kernel": "fused_topk", "score_kernel": "score", "topk_kernel": "topk",
         "psort_scatter_kernel": "psort_scatter", "psort_scan_kernel": "psort_scan",
         "scan_impl": "psort_scan", "init_lookback_scan_state": "psort_scan_init"}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return None


def per_kernel(d, counter):
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != counter:
                    continue
                k = short(row["Kernel_Name"])
                if k:
                    acc[k].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def durations(d):
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Name"])
                if k:
                    out[k] = float(row["AverageNs"])
    return out


def kernel_csv(d, counter, out):
    """Per-kernel mean of one counter (KiB) -> profiles/<round>/<tag>_pmc_*.csv"""
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == counter:
                    acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    with open(out, "w") as f:
        f.write("kernel,counter,dispatches,mean_value_KiB\n")
        for k in sorted(acc):
            f.write('"%s",%s,%d,%.3f\n' % (k, counter, len(acc[k]), sum(acc[k]) / len(acc[k])))


def main():
    tag, fdir, wdir = sys.argv[1:4]
    tdir = sys.argv[4] if len(sys.argv) > 4 else None
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    dur = durations(tdir) if tdir else {}
    rec = {}
    for k in sorted(set(fetch) | set(write)):
        f_raw = fetch.get(k, 0.0) * 1024.0
        w = write.get(k, 0.0) * 1024.0
        r = {"fetch_bytes_raw": f_raw, "fetch_bytes_corrected": 2.0 * f_raw,
             "write_bytes": w, "hbm_bytes_corrected": 2.0 * f_raw + w}
        if k in dur:
            r["rocprof_avg_ns"] = dur[k]
            r["hbm_GBps_corrected"] = r["hbm_bytes_corrected"] / dur[k]
        rec[k] = r
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = {}
    if os.path.exists(path):
        with open(path) as f:
            data = json.load(f)
    data[tag] = {"kernels": rec,
                 "step_hbm_bytes_per_launch": rec.get("step", {}).get("hbm_bytes_corrected"),
                 "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                           "KiB -> bytes, FETCH x2 gfx950 correction"}
    with open(path, "w") as f:
        json.dump(data, f, indent=1)
    rnd = os.environ.get("CF_ROUND", "r01")
    os.makedirs(os.path.join(ROOT, "profiles", rnd), exist_ok=True)
    kernel_csv(fdir, "FETCH_SIZE", os.path.join(ROOT, "profiles", rnd, tag + "_pmc_fetch.csv"))
    kernel_csv(wdir, "WRITE_SIZE", os.path.join(ROOT, "profiles", rnd, tag + "_pmc_write.csv"))
    print(json.dumps(data[tag], indent=1))


if __name__ == "__main__":
    main()
