#!/bin/bash
# Round-2: GBPR bias accumulators prefetched with the rows (cfg4 gradient).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "gbpr or group or bench_configs" tests > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
Q="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0"
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
run cfg4_a --config cfg4
run cfg2_a --config cfg2
run cfg4_b --config cfg4
echo ALL DONE
