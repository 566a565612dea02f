#!/bin/bash
# A/B on the cfg2 bench (kernel averages from the in-bench HIP-event
# profiler): default build with both grad paths, then every experimental build
# under build/variants/*.
set -o pipefail
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 200 --warmup 20 --no-cpu-baseline}
timeout -k 10 300 python bench.py $ARGS > gpurun_out/var_default.json 2> gpurun_out/var_default.err || exit 1
timeout -k 10 300 python bench.py $ARGS --grad-path 1 > gpurun_out/var_generic.json 2> gpurun_out/var_generic.err || exit 1
for lib in collaborativefilteringusingtensorflow_amd/build/variants/*/libcf_engine.so; do
  [ -f "$lib" ] || continue
  v=$(basename $(dirname $lib))
  CF_ENGINE_LIB=$PWD/$lib timeout -k 10 300 python bench.py $ARGS > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { echo "variant $v failed"; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/var_*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    k = r["kernels"]
    print(f.split("var_")[1][:-5], "ms/step %.4f" % r["ms_per_step"], " ".join("%s=%.1fus" % (n, v["avg_us"]) for n, v in k.items()))
PY
