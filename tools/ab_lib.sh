#!/bin/bash
# A/B of the default build against build/variants/* on the cfg2 bench, each
# with extra option sets: VARIANT_OPTS="name:args;name:args"
set -o pipefail
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 200 --warmup 20 --no-cpu-baseline --no-ndcg}
OPTS=${VARIANT_OPTS:-"base:"}
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  CF_ENGINE_LIB=$lib timeout -k 10 200 python bench.py $ARGS "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "variant $n failed"; tail -5 gpurun_out/ab_$n.err; exit 1; }
}
rm -f gpurun_out/ab_*.json
IFS=';' read -ra OS <<< "$OPTS"
for lib in collaborativefilteringusingtensorflow_amd/build/libcf_engine.so collaborativefilteringusingtensorflow_amd/build/variants/*/libcf_engine.so; do
  [ -f "$lib" ] || continue
  v=$(basename $(dirname $lib)); [ "$v" = build ] && v=default
  for o in "${OS[@]}"; do
    on=${o%%:*}; oa=${o#*:}
    run ${v}_$on $PWD/$lib $oa || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    k = r.get("kernels", {})
    print("%-22s ms/step %.4f " % (f.split("ab_")[1][:-5], r["ms_per_step"]), " ".join("%s=%.1fus" % (n, v["avg_us"]) for n, v in k.items() if isinstance(v, dict) and v["launches"] > 1))
PY
