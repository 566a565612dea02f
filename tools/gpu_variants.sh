#!/bin/bash
# A/B on the cfg2 bench (kernel averages from the in-bench HIP-event
# profiler): default build (both grad paths, in-order and overlapped prep,
# profiler off), then every experimental build under build/variants/*
# (in-order prep so kernel times are standalone).
set -o pipefail
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 200 --warmup 20 --no-cpu-baseline --no-ndcg}
run() {  # name, extra args...
  local n=$1; shift
  timeout -k 10 300 python bench.py $ARGS "$@" > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err || { echo "variant $n failed"; tail -5 gpurun_out/var_$n.err; exit 1; }
}
run default
run noprof --no-profile
run stepwise --pipeline 0
run stepwise_noprof --pipeline 0 --no-profile
run generic --grad-path 1
run atomics --slot-max 1
run slot8 --slot-max 8
run slot128 --slot-max 128
for lib in collaborativefilteringusingtensorflow_amd/build/variants/*/libcf_engine.so; do
  [ -f "$lib" ] || continue
  v=$(basename $(dirname $lib))
  CF_ENGINE_LIB=$PWD/$lib run x_$v --prep-stream 0
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/var_*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    k = r.get("kernels", {})
    print("%-16s ms/step %.4f " % (f.split("var_")[1][:-5], r["ms_per_step"]), " ".join("%s=%.1fus" % (n, v["avg_us"]) for n, v in k.items()))
PY
