#!/bin/bash
# Round-2: how much of cfg2's draw / apply is the Zipf head (hot counters,
# hot slot rows)?  Separate launches (pipeline 0) at item skew 0.8 / 0.4 / 0.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02h
mkdir -p $OUT
Q="--steps 60 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0"
summ() {
python - "$1" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read())
k = r["kernels"]
print(sys.argv[1].split("/")[-1], "ms/step %.4f" % r["ms_per_step"], {n: round(v["avg_us"], 1) for n, v in k.items() if isinstance(v, dict) and v["launches"] > 1})
PY
}
run() { # name args
  local n=$1; shift
  timeout -k 10 300 python bench.py $Q "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -5 $OUT/$n.err; exit 1; }
  summ $OUT/$n.json
}
for z in 0.8 0.4 0.0; do
  run cfg2_p0_z$z --config cfg2 --pipeline 0 --zipf $z
  run cfg2_p1_z$z --config cfg2 --zipf $z
done
run cfg2_p0_hr4 --config cfg2 --pipeline 0 --hot-replicas 4
run cfg2_p0_hr8 --config cfg2 --pipeline 0 --hot-replicas 8
run cfg3_p0 --config cfg3 --pipeline 0
run cfg3_p0_z0 --config cfg3 --pipeline 0 --zipf 0
echo ALL DONE
