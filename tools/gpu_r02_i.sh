#!/bin/bash
# Round-2 owner lists (cf_set_option apply_list): full GPU suite, then A/B.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
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
for c in cfg2 cfg3 cfg4 cfg5; do
  run ${c}_scan --config $c --apply-list 0
  run ${c}_list --config $c --apply-list 1
done
run cfg2_p0_scan --config cfg2 --apply-list 0 --pipeline 0
run cfg2_p0_list --config cfg2 --apply-list 1 --pipeline 0
echo ALL DONE
