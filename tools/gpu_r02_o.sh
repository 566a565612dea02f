#!/bin/bash
# (1) draw attribution: the default build against build/variants/noret_all
#     (every count atomic non-returning) with separate draw launches
#     (pipeline 0, pos_sort 0: the variant's ranks are all zero);
# (2) rocprof kernel trace + FETCH/WRITE passes of the default cfg2 line at
#     one batch size (pos_sort auto)
set -o pipefail
export PYTHONUNBUFFERED=1
VARIANT_OPTS="p0:--pipeline 0 --pos-sort 0" BENCH_ARGS="--steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0" bash tools/ab_lib.sh || exit 1
TAG=cfg2_b524288_psort BENCH_ARGS="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0" bash tools/gpu_profile.sh || exit 1
